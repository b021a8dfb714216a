"""Host-side cost of one eager training step vs its GPU time (is the GPU ever starved?).

    python tools/cpu_overhead.py [--batch 512] [--steps 20]
Prints the wall time to ISSUE the steps (no synchronisation) and the wall time until the GPU is done."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO  # noqa: E402
from proteinbert_pytorch_replication_amd.models import ProteinBERT  # noqa: E402
from proteinbert_pytorch_replication_amd.train.optim import FusedAdam  # noqa: E402
from proteinbert_pytorch_replication_amd.train.step import PretrainStep  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=512)
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda")
torch.manual_seed(0)
m = ProteinBERT(sequences_length=512, num_annotations=8943, local_dim=128, global_dim=512, key_dim=64, num_heads=4,
                num_blocks=6, device=dev, backend="hip")
opt = FusedAdam(m.parameters(), lr=2e-4)
step = PretrainStep(m, opt)
gen = SyntheticUniRefGO(512, 8943, a.batch, dev, seed=1)
for _ in range(5):
    step(*gen.next_batch())
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.steps):
    step(*gen.next_batch())
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"issue {1000 * (t1 - t0) / a.steps:.3f} ms/step   complete {1000 * (t2 - t0) / a.steps:.3f} ms/step", flush=True)
if os.environ.get("PBX_CPROFILE"):
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        step(*gen.next_batch())
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(35)
