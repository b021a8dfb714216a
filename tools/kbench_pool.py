"""Time the attention-pool backward kernels in isolation (paper config shapes): attn_bwd2 (Wv in LDS,
dv applied per streamed fragment) vs attn_bwd4 (weight-stationary, csrc/pool_bwd.hip) at several
tiles-per-workgroup, against a device copy of the same bytes.   python tools/kbench_pool.py [--B 512]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from proteinbert_pytorch_replication_amd.ops import _lib  # noqa: E402
from proteinbert_pytorch_replication_amd.ops import local_track as lt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=512)
ap.add_argument("--L", type=int, default=512)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
B, L, C, NJ = a.B, a.L, 128, 512
dev = torch.device("cuda")
st = _lib.stream_ptr(dev)
bf = torch.bfloat16


def timeit(fn, n=a.iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000.0


TW = (L + 31) // 32
TWG = 2 * ((L + 63) // 64)
s2 = torch.randn(B, L, C, device=dev).to(bf)
T2 = (L + 31) // 32
st2 = torch.zeros(B, T2, 2, device=dev)
st2[..., 1] = 32 * C
g2 = torch.ones(L, C, device=dev)
wv = (torch.randn(NJ, C, device=dev) * 0.05).to(bf)
gfrag = torch.randn(B, TWG, NJ * 32, device=dev).to(bf)
dh2_in = torch.randn(B, L, C, device=dev).to(bf)
dv = torch.randn(B, NJ, device=dev) * 1e-2
dh2 = torch.empty_like(s2)
sums2 = torch.empty(B, 4 * TW, 2, device=dev)
wvt = lt.wvt_frag(wv)
nbytes = gfrag.numel() * 2 + 3 * s2.numel() * 2
print(f"B={B} L={L}: {nbytes / 1e6:.0f} MB moved per call (GELU' fragments + dh2_in + s2 + dh2)")
us = timeit(lambda: _lib.call("pbx_attn_bwd2", gfrag.data_ptr(), s2.data_ptr(), st2.data_ptr(), g2.data_ptr(),
                              dh2_in.data_ptr(), dv.data_ptr(), L, wv.data_ptr(), dh2.data_ptr(), sums2.data_ptr(), B, L,
                              NJ, 1e-5, st))
print(f"attn_bwd2            {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s", flush=True)
for tpw in (0, 1, 2, 4, 8, 16):
    us = timeit(lambda: _lib.call("pbx_attn_bwd4", gfrag.data_ptr(), s2.data_ptr(), st2.data_ptr(), g2.data_ptr(),
                                  dh2_in.data_ptr(), dv.data_ptr(), wvt.data_ptr(), dh2.data_ptr(), sums2.data_ptr(),
                                  B, L, NJ, 1e-5, tpw, st))
    print(f"attn_bwd4 tpw={tpw:2d}      {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s", flush=True)
flat = gfrag.view(-1)
dst = torch.empty_like(flat)
us = timeit(lambda: dst.copy_(flat))
print(f"copy GELU' fragments {us:8.1f} us  {2 * flat.numel() * 2 / us / 1e6:6.2f} TB/s (read + write)")
