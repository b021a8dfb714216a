"""Per-kernel timing of the fused local-track kernels on the paper config (B=256, L=512).

    python tools/kbench.py [--B 256] [--L 512] [--iters 20]

Prints us/call and effective TFLOP/s (MFMA FLOPs the kernel performs) for each launcher, with
variants (tile sizes) where the launcher exposes them.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from proteinbert_pytorch_replication_amd.ops import _lib  # noqa: E402
from proteinbert_pytorch_replication_amd.ops import local_track as lt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=256)
ap.add_argument("--L", type=int, default=512)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
B, L, C, KS, dil = a.B, a.L, 128, 9, 5
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


def report(name, us, flops=None, bytes_=None):
    extra = ""
    if flops:
        extra += f"  {flops / us / 1e6:8.1f} TFLOP/s"
    if bytes_:
        extra += f"  {bytes_ / us / 1e6:8.2f} TB/s"
    print(f"{name:40s} {us:9.1f} us{extra}", flush=True)


x = (torch.randn(B, L, C, device=dev) * 0.5).to(bf)
w = torch.randn(C, C, KS, device=dev) * 0.03
wpn, wtn = lt.pack_conv(w)
wpw, wtw = lt.pack_conv(w)
bias = torch.zeros(C, device=dev)
gb = torch.zeros(B, C, device=dev)
act = lambda: torch.empty_like(x)  # noqa: E731
pre_n, pre_w, s1 = act(), act(), act()
conv_flops = 2 * 2 * B * L * C * C * KS
for BM in (256, 128):
    T = (L + BM - 1) // BM
    stt = torch.empty(B, T, 2, device=dev)
    us = timeit(lambda: _lib.call("pbx_conv_fwd", x.data_ptr(), wpn.data_ptr(), wpw.data_ptr(), bias.data_ptr(),
                                  bias.data_ptr(), gb.data_ptr(), pre_n.data_ptr(), pre_w.data_ptr(), s1.data_ptr(),
                                  stt.data_ptr(), B, L, KS, dil, BM, st))
    report(f"conv_fwd BM={BM}", us, conv_flops, 4 * x.numel() * 2)
    dx, dpn, dpw = act(), act(), act()
    us = timeit(lambda: _lib.call("pbx_conv_dgrad", s1.data_ptr(), pre_n.data_ptr(), pre_w.data_ptr(),
                                  wtn.data_ptr(), wtw.data_ptr(), dx.data_ptr(), dpn.data_ptr(), dpw.data_ptr(), B, L,
                                  KS, dil, BM, st))
    report(f"conv_dgrad BM={BM}", us, conv_flops, 6 * x.numel() * 2)
dw0 = torch.zeros(C, C, KS, device=dev)
dw1 = torch.zeros(C, C, KS, device=dev)
db0 = torch.zeros(C, device=dev)
db1 = torch.zeros(C, device=dev)
for R in (32, 64, 128):
    slab = torch.empty(R, 2, KS, C, C, device=dev)
    bslab = torch.empty(R, 2, C, device=dev)
    us = timeit(lambda: _lib.call("pbx_wgrad", pre_n.data_ptr(), pre_w.data_ptr(), x.data_ptr(), slab.data_ptr(),
                                  bslab.data_ptr(), dw0.data_ptr(), dw1.data_ptr(), db0.data_ptr(), db1.data_ptr(), B,
                                  L, KS, dil, 2, R, 1, st))
    report(f"conv wgrad+reduce R={R}", us, conv_flops)
