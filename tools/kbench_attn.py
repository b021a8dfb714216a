"""Time the attention-pool kernels (ln_attn_fwd, attn_bwd) and the LN kernels in isolation on the
paper config, for several workgroup sizes.   python tools/kbench_attn.py [--B 256] [--L 512]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from proteinbert_pytorch_replication_amd.ops import _lib  # noqa: E402
from proteinbert_pytorch_replication_amd.ops import local_track as lt  # noqa: E402,F401

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=256)
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


s2 = (torch.randn(B, L, C, device=dev)).to(bf)
T2 = (L + 31) // 32
st2 = torch.zeros(B, T2, 2, device=dev)
st2[..., 1] = 32 * C     # mean 0, var 1
g2 = torch.ones(L, C, device=dev)
be2 = torch.zeros(L, C, device=dev)
wv = (torch.randn(NJ, C, device=dev) * 0.05).to(bf)
h2 = torch.empty_like(s2)
vpart = torch.empty(B, (L + 63) // 64, NJ, device=dev)
flops = 2 * B * L * C * NJ
for nw in (4, 8):
    us = timeit(lambda: _lib.call("pbx_ln_attn_fwd", s2.data_ptr(), st2.data_ptr(), g2.data_ptr(), be2.data_ptr(),
                                  wv.data_ptr(), h2.data_ptr(), vpart.data_ptr(), B, L, NJ, nw, 1e-5, st))
    print(f"ln_attn_fwd nw={nw:2d}  {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s  "
          f"{(2 * s2.numel() * 2) / us / 1e6:6.2f} TB/s", flush=True)
dv = torch.randn(B, NJ, device=dev) * 1e-3
dh2 = torch.empty_like(s2)
sums2 = torch.empty(B, (L + 31) // 32, 2, device=dev)
for nw in (4, 8):
    us = timeit(lambda: _lib.call("pbx_attn_bwd", h2.data_ptr(), s2.data_ptr(), st2.data_ptr(), g2.data_ptr(), 0,
                                  dv.data_ptr(), (L + 31) // 32 * 32, wv.data_ptr(), dh2.data_ptr(), sums2.data_ptr(),
                                  B, L, NJ, nw, 1e-5, st))
    print(f"attn_bwd nw={nw}  {us:8.1f} us  {2 * flops / us / 1e6:7.1f} TF/s  "
          f"{(3 * s2.numel() * 2) / us / 1e6:6.2f} TB/s", flush=True)
# pure streaming reference: copy s2 -> h2 (bandwidth ceiling for a read+write of this tensor)
us = timeit(lambda: h2.copy_(s2))
print(f"copy bf16 [B,L,C]      {us:8.1f} us  {(2 * s2.numel() * 2) / us / 1e6:6.2f} TB/s")
