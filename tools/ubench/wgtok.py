"""Time the first block's conv weight gradient: wgrad2 over the 128 embedding channels (full chip, as the
step's tail launch) vs wgrad_tok (token one-hot GEMM + E^T S), paper config shapes.
    python tools/ubench/wgtok.py [--B 512 --L 512]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from proteinbert_pytorch_replication_amd.ops import local_track as lt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=512)
ap.add_argument("--L", type=int, default=512)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
B, L = a.B, a.L
dev = torch.device("cuda")
torch.manual_seed(0)
E = torch.randn(26, 128, device=dev)
tok = torch.randint(0, 26, (B, L), device=dev)
x = E.to(torch.bfloat16)[tok].contiguous()
dpn = torch.randn(B, L, 128, device=dev).to(torch.bfloat16)
dpw = torch.randn(B, L, 128, device=dev).to(torch.bfloat16)


def outs():
    return [(torch.zeros(128, 128, 9, device=dev), torch.zeros(128, device=dev)) for _ in range(2)]


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


o1, o2 = outs(), outs()
us2 = timeit(lambda: lt._wgrad(dpn, dpw, x, 9, 5, 2, B, L, o1, True))
ust = timeit(lambda: lt._wgrad_tok(dpn, dpw, tok, E, 5, B, L, o2))
print(f"B={B} L={L}: wgrad2 (full chip) {us2:7.1f} us   wgrad_tok {ust:7.1f} us", flush=True)
o1, o2 = outs(), outs()
lt._wgrad(dpn, dpw, x, 9, 5, 2, B, L, o1, True)
lt._wgrad_tok(dpn, dpw, tok, E, 5, B, L, o2)
torch.cuda.synchronize()
for (a1, b1), (a2, b2) in zip(o1, o2):
    print("max |dW diff| / |dW|:", float((a1 - a2).abs().max() / a1.abs().max()),
          " db:", float((b1 - b2).abs().max() / b1.abs().max()))
