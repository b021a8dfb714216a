"""Host-code sanitizers (race detection / memory errors) on the native threaded batch
builder ``ops/csrc/pbx_loader.cpp``: the library source is compiled together with a C++ driver
(``tools/sanitize/loader_driver.cpp``) under AddressSanitizer + UndefinedBehaviorSanitizer and,
separately, ThreadSanitizer (the worker ring: atomic batch claiming, slot hand-off, shutdown with
workers mid-batch), and run over a small .pbxds store.  Any sanitizer report fails the test.
GPU sanitizers (GPU ASan / xnack+) are not available on the MI355X pool; the HIP kernels are checked by
the GPU numerics tests and host-side shape checks instead."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from proteinbert_pytorch_replication_amd.data.store import ProteinStoreWriter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "proteinbert_pytorch_replication_amd", "ops", "csrc", "pbx_loader.cpp")
DRIVER = os.path.join(ROOT, "tools", "sanitize", "loader_driver.cpp")
A = 300


@pytest.fixture(scope="module")
def store(tmp_path_factory):
    d = tmp_path_factory.mktemp("san")
    path = str(d / "s.pbxds")
    rng = np.random.default_rng(0)
    w = ProteinStoreWriter(path, ["GO:%07d" % i for i in range(A)])
    for i in range(37):
        n = int(rng.integers(5, 150))
        w.append_mask("P%d" % i, "".join(rng.choice(list("ACDEFGHIKLMNPQRSTVWY"), n)), rng.random(A) < 0.05)
    w.close()
    return path


def _build_and_run(tmp_path, store, flags, env_extra):
    cxx = shutil.which(os.environ.get("CXX", "g++"))
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "driver")
    cmd = [cxx, "-O1", "-g", "-std=c++17", "-fno-omit-frame-pointer", "-pthread", *flags, "-I",
           os.path.dirname(SRC), SRC, DRIVER, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        if "sanitizer" in r.stderr.lower() and ("cannot find" in r.stderr or "not supported" in r.stderr):
            pytest.skip(f"sanitizer runtime unavailable: {r.stderr[-300:]}")
        raise AssertionError(r.stderr)
    env = dict(os.environ, **env_extra)
    r = subprocess.run([exe, store, str(A)], capture_output=True, text=True, env=env, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "Sanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert out.startswith("ok ")
    return out.split()[1]


def test_loader_asan_ubsan(tmp_path, store):
    _build_and_run(tmp_path, store, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
                   {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0"})


def test_loader_tsan(tmp_path, store):
    _build_and_run(tmp_path, store, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1"})


def test_loader_sanitized_output_is_deterministic(tmp_path, store):
    """The checksum of every batch does not depend on the sanitizer build (same order, same crops)."""
    a = _build_and_run(tmp_path, store, [], {})
    b = _build_and_run(tmp_path, store, ["-fsanitize=address,undefined"], {"ASAN_OPTIONS": "detect_leaks=1"})
    assert a == b
