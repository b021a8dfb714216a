"""Per-wave phase cycles of conv_dgrad4<FIN> (csrc/conv4.hip built with -DPBX_STAMPS): prologue (LN1 finalize
+ dpre staging), MFMA loop, dx epilogue; B = 1024, L = 512 (4096 workgroups of 4 waves).
    PBX_HIP_LIB=tools/ubench/abl/libpbx_stamps.so python tools/ubench/dgradstamps.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from proteinbert_pytorch_replication_amd.ops import _lib, local_track as lt  # noqa: E402

B, L, C, KS, dil = 1024, 512, 128, 9, 5
dev = torch.device("cuda")
st = _lib.stream_ptr(dev)
torch.manual_seed(0)
bf = torch.bfloat16
T1 = (L + lt.BM1 - 1) // lt.BM1
TS1 = (L + 1) // 2
dh1, s1, gdn, gdw = ((torch.randn(B, L, C, device=dev) * 0.5).to(bf) for _ in range(4))
st1 = torch.zeros(B, T1, 2, device=dev)
st1[..., 1] = lt.BM1 * C * 0.25
sums1 = torch.randn(B, TS1, 2, device=dev) * 0.01
g1 = torch.ones(L, C, device=dev)
w = torch.randn(C, C, KS, device=dev) * 0.03
_, wt = lt.pack_conv(w)
dx, dpn, dpw = (torch.empty_like(dh1) for _ in range(3))
dgb = torch.zeros(B, C, device=dev)
run = lambda: _lib.call("pbx_conv_dgrad4f", dh1.data_ptr(), s1.data_ptr(), st1.data_ptr(), T1, lt.BM1,  # noqa
                        sums1.data_ptr(), TS1, g1.data_ptr(), gdn.data_ptr(), gdw.data_ptr(), wt.data_ptr(),
                        wt.data_ptr(), dx.data_ptr(), dpn.data_ptr(), dpw.data_ptr(), dgb.data_ptr(), B, L, KS, dil,
                        1e-5, st)
for _ in range(3):
    run()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
run()
e1.record()
torch.cuda.synchronize()
n = 4096 * 4 * 4
buf = (ctypes.c_ulonglong * n)()
assert _lib.lib().pbx_dgrad_stamps_read(buf, n) == 0
t = torch.tensor(list(buf), dtype=torch.float64).view(4096, 4, 4)
print(f"conv_dgrad4<FIN> {e0.elapsed_time(e1) * 1000:.1f} us (instrumented)")
for i, name in enumerate(["prologue", "MFMA loop", "epilogue"]):
    v = t[:, :, i]
    print(f"  {name:10s} mean {v.mean():8.0f} cycles/WG-wave  (p10 {v.quantile(0.1):.0f}, p90 {v.quantile(0.9):.0f})")
