"""GPU probe: is the fused pretraining step bitwise repeatable when the caching allocator hands out dirty
memory?  Runs the same step (fixed weights, fixed batch) several times, filling the allocator with NaN
buffers between runs, and records every conv forward's inputs and outputs (local_track.conv_fwd) and all
parameter gradients; prints the first difference.

    python tools/probe_conv_det.py [--fold 0|1] [--runs 4]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
from proteinbert_pytorch_replication_amd.models import ProteinBERT
from proteinbert_pytorch_replication_amd.ops import local_track, streams
from proteinbert_pytorch_replication_amd.train.optim import FusedAdam
from proteinbert_pytorch_replication_amd.train.step import PretrainStep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fold", type=int, default=0)
    ap.add_argument("--runs", type=int, default=4)
    ap.add_argument("--L", type=int, default=256)
    ap.add_argument("--blocks", type=int, default=2)
    a = ap.parse_args()
    local_track.EMBED_FOLD = bool(a.fold)
    L, A = a.L, 512
    X, Y, W = SyntheticUniRefGO(L, A, 6, "cuda", seed=9).next_batch()
    rec = []
    orig = local_track.conv_fwd

    def spy(x, wpn, wpw, bn, bw, gb, pre_n, pre_w, s1, stats, B, L_, KS, dil, stream, *args, **kw):
        xin = x.clone() if x.dtype != torch.int64 else x.clone()
        orig(x, wpn, wpw, bn, bw, gb, pre_n, pre_w, s1, stats, B, L_, KS, dil, stream, *args, **kw)
        torch.cuda.synchronize()
        rec[-1].append({"x": xin, "gb": gb.clone(), "s1": s1.clone(), "stats": stats.clone(),
                        "pre_n": None if pre_n is None else pre_n.clone(),
                        "pre_w": None if pre_w is None else pre_w.clone(), "dil": dil})

    local_track.conv_fwd = spy
    grads = []
    for run in range(a.runs):
        junk = [torch.full((64 << 20,), float("nan"), device="cuda") for _ in range(8)]
        del junk
        rec.append([])
        torch.manual_seed(0)
        m = ProteinBERT(sequences_length=L, num_annotations=A, local_dim=128, global_dim=512, key_dim=64,
                        num_heads=4, num_blocks=a.blocks, device="cuda", backend="hip")
        step = PretrainStep(m, FusedAdam(m.parameters(), lr=1e-3))
        step.optimizer.zero_grad()
        step.loss(X, Y, W).backward()
        streams.join()
        torch.cuda.synchronize()
        grads.append({n: p.grad.detach().float().clone() for n, p in m.named_parameters() if p.grad is not None})
        del step, m
    bad = 0
    for run in range(1, a.runs):
        for i, (u, v) in enumerate(zip(rec[0], rec[run])):
            for k in ("x", "gb", "s1", "stats", "pre_n", "pre_w"):
                if u[k] is None:
                    continue
                if not torch.equal(u[k], v[k]):
                    d = (u[k].float() - v[k].float()).abs()
                    nz = torch.nonzero(d.reshape(-1) != 0)
                    print(f"run {run} conv call {i} (dil {u['dil']}) {k}: {nz.numel()} differ, max {d.max().item():.3e},"
                          f" first flat idx {nz[:5].flatten().tolist()} shape {tuple(u[k].shape)}")
                    bad += 1
        for n in grads[0]:
            if not torch.equal(grads[0][n], grads[run][n]):
                print(f"run {run} grad {n}: max diff {(grads[0][n] - grads[run][n]).abs().max().item():.3e}")
                bad += 1
    print("conv calls per run:", len(rec[0]), "differences:", bad)


if __name__ == "__main__":
    main()
