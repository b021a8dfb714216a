"""CPU: the persistent conv forward (csrc/conv5.hip) issues its weight-fragment loads in inline asm, invisible
to the compiler; a register copy of such a load before the kernel's own vmcnt wait retires it reads a stale
value and lets the late write corrupt the register's new owner (round 6: a persistent data-gradient
prototype did exactly that to an address register and faulted, profiles/r6/conv_dgrad5_attempts.txt).
Compile for gfx950 and check the ISA with tools/asm_hazards.py (forward dataflow over the in-order
vector-memory queue)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "proteinbert_pytorch_replication_amd", "ops", "csrc")
sys.path.insert(0, os.path.join(ROOT, "tools"))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src,kernels", [("conv5.hip", ["conv_fwd5_kernelILb1", "conv_fwd5_kernelILb0"])])
def test_no_inflight_load_register_hazards(tmp_path, src, kernels):
    import asm_hazards
    from proteinbert_pytorch_replication_amd.ops import build
    out = tmp_path / (src + ".s")
    flags = [f for f in build.hip_flags() if f not in ("-fPIC",)]
    subprocess.run([HIPCC, *flags, "--cuda-device-only", "-S", "-o", str(out), os.path.join(CSRC, src)],
                   check=True, capture_output=True)
    for k in kernels:
        assert asm_hazards.main(str(out), k) == 0, k
