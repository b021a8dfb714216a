"""Per-wave phase cycles of conv_dgrad5 (csrc/conv5.hip built with -DPBX_STAMPS), summed over each
workgroup's tiles; B = 1024, L = 512 (4096 tiles over 256 persistent workgroups).
    PBX_HIP_LIB=tools/ubench/abl/libpbx_stamps5.so python tools/ubench/dgrad5stamps.py"""
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
extra = (torch.empty(B, 4, device=dev).data_ptr(),)
run = lambda: _lib.call("pbx_conv_dgrad5f", dh1.data_ptr(), s1.data_ptr(), st1.data_ptr(), T1, lt.BM1,  # noqa
                        sums1.data_ptr(), TS1, g1.data_ptr(), gdn.data_ptr(), gdw.data_ptr(), wt.data_ptr(),
                        wt.data_ptr(), dx.data_ptr(), dpn.data_ptr(), dpw.data_ptr(), dgb.data_ptr(), *extra, B, L, KS, dil,
                        1e-5, st)
for _ in range(3):
    run()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
run()
e1.record()
torch.cuda.synchronize()
n = 256 * 16 * 8
buf = (ctypes.c_ulonglong * n)()
assert _lib.lib().pbx_dgrad5_stamps_read(buf, n) == 0
t = torch.tensor(list(buf), dtype=torch.float64).view(256, 16, 8)
ntile = B * ((L + 127) // 128) / 256
print(f"conv_dgrad5 {e0.elapsed_time(e1) * 1000:.1f} us (instrumented); per-tile means over 256 workgroups")
names_c = ["MFMA loop", "dx epilogue", "wait P", "", "", "", "", "prologue wait P0"]
names_p = ["stage", "wait P", "", "", "", "", "stage(0)", "wait P0"]
for w, names in ((0, names_c), (4, names_p), (7, names_p)):
    print(f" wave {w}:")
    for k, nm in enumerate(names):
        if nm:
            v = t[:, w, k] / (1 if k >= 6 else ntile)
            print(f"   {nm:18s} {v.mean():9.0f}  (p10 {v.quantile(0.1):.0f}, p90 {v.quantile(0.9):.0f})")
