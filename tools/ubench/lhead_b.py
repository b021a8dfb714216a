"""Time the reference-semantics local head at the headline shapes: the one-launch fused kernel vs the
five-pass form (ops/global_track.py local_head_forward, LHEAD_FUSED).
    python tools/ubench/lhead_b.py [--B 1024 --L 512]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from proteinbert_pytorch_replication_amd.ops import global_track as gt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=1024)
ap.add_argument("--L", type=int, default=512)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda")
torch.manual_seed(0)
B, L, V = a.B, a.L, 26
h = torch.randn(B, L, 128, device=dev).to(torch.bfloat16)
wo, bo = torch.randn(V, 128, device=dev) * 0.1, torch.randn(V, device=dev)
y = torch.randint(0, V, (B, L), device=dev)
w = torch.ones(B, L, device=dev)


def run():
    loss = torch.zeros(1, device=dev)
    return gt.local_head_forward(h, wo, bo, y, w, loss), loss


res = {}
for fused in (True, False):
    gt.LHEAD_FUSED = fused
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        out = run()
    e1.record()
    torch.cuda.synchronize()
    res[fused] = out
    print(f"B={B} L={L} fused={fused}: {e0.elapsed_time(e1) / a.iters * 1000:.1f} us", flush=True)
(d1, z1, _), l1 = res[True]
(d2, z2, _), l2 = res[False]
print("max |dh diff|:", float((d1.float() - d2.float()).abs().max()), " loss:", float(l1), float(l2))
