"""Per-wave phase cycle totals of the pool backward (csrc/pool.hip built with -DPBX_STAMPS:
tools/ubench/build_flags.sh stamps -DPBX_STAMPS=1): wait for the item's h2 / dv loads, main loop, epilogue.
    PBX_HIP_LIB=tools/ubench/abl/libpbx_stamps.so python tools/ubench/poolstamps.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from proteinbert_pytorch_replication_amd.ops import _lib  # noqa: E402
from proteinbert_pytorch_replication_amd.ops import local_track  # noqa: E402,F401

B, L, C, NJ = 1024, 512, 128, 512
dev = torch.device("cuda")
st = _lib.stream_ptr(dev)
TW = (L + 31) // 32
h2 = torch.randn(B, L, C, device=dev).to(torch.bfloat16)
g2, be2 = torch.ones(L, C, device=dev), torch.zeros(L, C, device=dev)
wv = (torch.randn(NJ, C, device=dev) * 0.1).to(torch.bfloat16)
dh2_in = torch.randn(B, L, C, device=dev).to(torch.bfloat16)
dv = torch.randn(B, NJ, device=dev) * 1e-2
dh2 = torch.empty_like(h2)
sums2 = torch.empty(B, TW, 2, device=dev)
run = lambda: _lib.call("pbx_pool_bwd", h2.data_ptr(), g2.data_ptr(), be2.data_ptr(), dh2_in.data_ptr(),  # noqa
                        dv.data_ptr(), 1, wv.data_ptr(), dh2.data_ptr(), sums2.data_ptr(), B, L, NJ, st)
for _ in range(3):
    run()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
run()
e1.record()
torch.cuda.synchronize()
n = 256 * 64 * 8 * 4
buf = (ctypes.c_ulonglong * n)()
assert _lib.lib().pbx_pool_stamps_read(buf, n) == 0
t = torch.tensor(list(buf), dtype=torch.float64).view(-1, 4)
t = t[t[:, 3] > 0]
items = t[:, 3]
print(f"pool_bwd {e0.elapsed_time(e1) * 1000:.1f} us; {t.shape[0]} waves, {items.mean():.1f} items each")
for i, name in enumerate(["wait h2/dv", "main loop", "epilogue"]):
    per = t[:, i] / items
    print(f"  {name:12s} {per.mean():9.0f} cycles/item (min {per.min():.0f}, max {per.max():.0f})  "
          f"total/wave {t[:, i].mean():10.0f}")
