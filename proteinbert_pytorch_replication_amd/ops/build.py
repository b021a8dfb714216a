"""Build the native libraries in-tree.

* ``libpbx_hip.so``   - every ``csrc/*.hip`` kernel file, compiled by hipcc for
  gfx950 only (``--offload-arch=gfx950``), linked into one shared object that
  :mod:`._lib` loads with ctypes.  No hipify, no torch extension machinery:
  each file is plain HIP C++ exposing ``extern "C"`` launchers that take raw
  device pointers and a ``hipStream_t`` (torch's current stream), so every
  launch is capturable in a hipGraph.
* ``libpbx_hip_exact.so`` - the same sources with ``-DPBX_GELU_EXACT=1``: every fused
  GELU / GELU' evaluates the erf form (A&S 7.1.26, |err| <= 1.5e-7) instead of the
  fitted logistic core.  :mod:`._lib` loads it when ``PBX_GELU=exact`` (or the
  ``kernel.gelu=exact`` config key) selects reference-exact activations.
* ``libpbx_host.so``  - host-only C++ runtime pieces (``csrc/*.cpp``: the
  threaded batch builder), compiled with g++.

Usage: ``python -m proteinbert_pytorch_replication_amd.ops.build [-v] [--force]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
from typing import List

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD_DIR = os.path.join(HERE, "_build")
HIP_LIB = os.path.join(HERE, "libpbx_hip.so")
HIP_LIB_EXACT = os.path.join(HERE, "libpbx_hip_exact.so")
# variant -> (extra hipcc flags, library path)
VARIANTS = {"fitted": ([], HIP_LIB), "exact": (["-DPBX_GELU_EXACT=1"], HIP_LIB_EXACT)}
HOST_LIB = os.path.join(HERE, "libpbx_host.so")
ARCH = "gfx950"


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build the HIP kernels)")


def _newer(target: str, deps: List[str]) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def _run(cmd: List[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose and r.stderr.strip():
        print(r.stderr, file=sys.stderr)


def hip_flags() -> List[str]:
    # -fno-slp-vectorize: the SLP vectoriser packs adjacent scalar f32 ops into v_pk_*_f32, which cost
    # more than their scalar halves beside in-flight MFMAs on gfx950; explicitly packed code (f32x2
    # GELU cores of the VALU-bound pool epilogue) stays packed.  +1.4 % on the step, same-box A/B
    # (tools/gpu_scalar_ab.sh, profiles/r2_v8_scalar_ab.txt).
    return ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
            "-ffp-contract=fast-honor-pragmas", "-fno-slp-vectorize", "-Wno-unused-result", "-I", CSRC]


def build_hip(verbose: bool = False, force: bool = False, jobs: int = 8, variant: str = "fitted") -> str:
    hipcc = _hipcc()
    extra, lib = VARIANTS[variant]
    bdir = BUILD_DIR if variant == "fitted" else os.path.join(BUILD_DIR, variant)
    os.makedirs(bdir, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    objs = []
    # a change of compiler flags rebuilds every object (mtimes alone would keep the old code)
    stamp = os.path.join(bdir, "flags.txt")
    flags = " ".join([hipcc, *hip_flags(), *extra])
    if not os.path.exists(stamp) or open(stamp).read() != flags:
        force = True

    def compile_one(src: str) -> str:
        obj = os.path.join(bdir, os.path.basename(src) + ".o")
        if force or not _newer(obj, [src] + headers):
            _run([hipcc, *hip_flags(), *extra, "-c", src, "-o", obj], verbose)
        return obj

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(compile_one, srcs))
    if force or not _newer(lib, objs):
        tmp = lib + ".tmp"
        _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp, *objs], verbose)
        os.replace(tmp, lib)
    with open(stamp, "w") as f:
        f.write(flags)
    return lib


def build_host(verbose: bool = False, force: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.cpp")))
    if not srcs:
        return ""
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    if force or not _newer(HOST_LIB, srcs + headers):
        cxx = os.environ.get("CXX", "g++")
        tmp = HOST_LIB + ".tmp"
        _run([cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-I", CSRC, "-o", tmp, *srcs], verbose)
        os.replace(tmp, HOST_LIB)
    return HOST_LIB


def build_all(verbose: bool = False, force: bool = False, jobs: int = 8) -> None:
    for v in VARIANTS:
        build_hip(verbose, force, jobs, v)
    build_host(verbose, force)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=8)
    a = ap.parse_args()
    build_all(a.verbose, a.force, a.jobs)
    print(HIP_LIB)


if __name__ == "__main__":
    main()
