"""Per-wave phase cycles of conv_fwd3 (csrc/conv2.hip built with -DPBX_STAMPS): x-tile staging, MFMA loop,
epilogue; B = 1024, L = 512 (4096 workgroups; the first 4096 are recorded).
    PBX_HIP_LIB=tools/ubench/abl/libpbx_stamps.so python tools/ubench/convstamps.py"""
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
x = (torch.randn(B, L, C, device=dev) * 0.5).to(torch.bfloat16)
w = torch.randn(C, C, KS, device=dev) * 0.03
wp, _ = lt.pack_conv(w)
bias = torch.randn(C, device=dev) * 0.1
gb = torch.randn(B, C, device=dev) * 0.1
pre_n, pre_w, s1 = (torch.empty_like(x) for _ in range(3))
stt = torch.empty(B, (L + 127) // 128, 2, device=dev)
run = lambda: lt.conv_fwd(x, wp, wp, bias, bias, gb, pre_n, pre_w, s1, stt, B, L, KS, dil, st)  # noqa: E731
for _ in range(3):
    run()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
run()
e1.record()
torch.cuda.synchronize()
n = 4096 * 8 * 4
buf = (ctypes.c_ulonglong * n)()
assert _lib.lib().pbx_conv_stamps_read(buf, n) == 0
t = torch.tensor(list(buf), dtype=torch.float64).view(4096, 8, 4)
print(f"conv_fwd3 {e0.elapsed_time(e1) * 1000:.1f} us (instrumented)")
for i, name in enumerate(["x staging", "MFMA loop", "epilogue"]):
    v = t[:, :, i]
    print(f"  {name:10s} mean {v.mean():8.0f} cycles/WG-wave  (p10 {v.quantile(0.1):.0f}, p90 {v.quantile(0.9):.0f})")
t0 = t[:, 0, 3]
span = t0.max() - t0.min()
print(f"  WG start spread {span:.0f} cycles; per-CU WGs ~16 -> ~{span / 16:.0f} cycles per WG slot")
