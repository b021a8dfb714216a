import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE_DIR = "/root/reference/ProteinBERT"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def reference_modules():
    """The reference model file imports with torch alone."""
    if not os.path.exists(os.path.join(REFERENCE_DIR, "modules.py")):
        pytest.skip("reference not mounted")
    sys.path.insert(0, REFERENCE_DIR)
    try:
        import modules  # type: ignore
    finally:
        sys.path.remove(REFERENCE_DIR)
    return modules


def _exported_launchers():
    """Every ``PBX_EXPORT int pbx_*`` entry point of libpbx_hip.so (read from the HIP sources)."""
    import glob
    import re
    names = set()
    for f in glob.glob(os.path.join(ROOT, "proteinbert_pytorch_replication_amd", "ops", "csrc", "*.hip")):
        with open(f) as fh:
            names.update(re.findall(r"PBX_EXPORT\s+int\s+(pbx_\w+)\s*\(", fh.read()))
    return names


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """GPU runs: report which kernel launchers the session reached through ``_lib.call``.

    ``_lib.call`` caches a ctypes function object on first use, so the cache keys are exactly the
    launchers that ran.  Written to ``$PBX_LAUNCHER_REPORT`` when set (evidence under profiles/)."""
    mod = sys.modules.get("proteinbert_pytorch_replication_amd.ops._lib")
    if mod is None or not getattr(mod, "_FN", None):
        return
    import glob
    import re
    exported = _exported_launchers()
    called = set(mod._FN)
    pkg = os.path.join(ROOT, "proteinbert_pytorch_replication_amd")
    queries, native = set(), set()
    for f in glob.glob(os.path.join(pkg, "**", "*.py"), recursive=True):   # host-side shape queries
        with open(f) as fh:
            queries.update(re.findall(r"lib\(\)\.(pbx_\w+)\(", fh.read()))
    for f in glob.glob(os.path.join(pkg, "ops", "csrc", "*.hip")):            # launched by another launcher
        with open(f) as fh:
            native.update(re.findall(r'extern "C" int (pbx_\w+)\(', fh.read()))
    lines = [f"kernel launchers reached: {len(called & exported)} of {len(exported)} exported"]
    for n in sorted(exported - called):
        why = ("host shape query, no kernel" if n in queries else
               "called from another launcher's C code" if n in native else "NOT REACHED")
        lines.append(f"  not via _lib.call: {n} ({why})")
    for ln in lines:
        terminalreporter.write_line(ln)
    out = os.environ.get("PBX_LAUNCHER_REPORT")
    if out:
        with open(out, "w") as fh:
            fh.write("\n".join(lines) + "\n")
