"""Experiment: does running two independent half-batch training steps on two HIP streams beat one
full-batch step?  (Upper bound for splitting the encoder into two concurrently running micro-batches.)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO  # noqa: E402
from proteinbert_pytorch_replication_amd.models import ProteinBERT  # noqa: E402
from proteinbert_pytorch_replication_amd.train.optim import FusedAdam  # noqa: E402
from proteinbert_pytorch_replication_amd.train.step import PretrainStep  # noqa: E402

dev = torch.device("cuda")


def make(B, seed):
    torch.manual_seed(seed)
    m = ProteinBERT(sequences_length=512, num_annotations=8943, local_dim=128, global_dim=512, key_dim=64,
                    num_heads=4, num_blocks=6, device=dev, backend="hip")
    opt = FusedAdam(m.parameters(), lr=2e-4)
    return PretrainStep(m, opt), SyntheticUniRefGO(512, 8943, B, dev, seed=seed)


def run(pairs, steps=30):
    streams = [torch.cuda.Stream() for _ in pairs]
    for _ in range(3):
        for (st, g), s in zip(pairs, streams):
            with torch.cuda.stream(s):
                st(*g.next_batch())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        for (st, g), s in zip(pairs, streams):
            with torch.cuda.stream(s):
                st(*g.next_batch())
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1000


full = run([make(256, 0)])
print(f"one B=256 step: {full:.3f} ms", flush=True)
half1 = run([make(128, 1)])
print(f"one B=128 step: {half1:.3f} ms", flush=True)
two = run([make(128, 2), make(128, 3)])
print(f"two B=128 steps on two streams: {two:.3f} ms (vs {full:.3f} for B=256)", flush=True)
