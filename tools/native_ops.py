"""GPU probe: which PyTorch ops launch at::native / runtime kernels inside the headline training step?
Runs bench-shaped steps (B = 1024, L = 512, paper config) and prints, for one profiled step, every device
kernel whose name is not one of the in-tree HIP kernels together with the CPU-side op that launched it.

    python tools/native_ops.py [--batch 1024]
"""
import argparse
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO  # noqa: E402
from proteinbert_pytorch_replication_amd.models import ProteinBERT  # noqa: E402
from proteinbert_pytorch_replication_amd.train.optim import FusedAdam  # noqa: E402
from proteinbert_pytorch_replication_amd.train.step import PretrainStep  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1024)
ap.add_argument("--semantics", default="reference")
a = ap.parse_args()
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = ProteinBERT(sequences_length=512, num_annotations=8943, local_dim=128, global_dim=512, key_dim=64, num_heads=4,
                num_blocks=6, device=dev, backend="hip", semantics=a.semantics)
opt = FusedAdam(m.parameters(), lr=2e-4)
step = PretrainStep(m, opt)
gen = SyntheticUniRefGO(512, 8943, a.batch, dev, seed=1)
for _ in range(3):
    step(*gen.next_batch())
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    step(*gen.next_batch())
    torch.cuda.synchronize()
evs = prof.events()
n = 0
for e in evs:
    if e.device_type.name != "CUDA":
        continue
    name = e.name
    if "at::native" in name or "rocclr" in name or "Memcpy" in name or "Memset" in name:
        parent = e.cpu_parent
        chain = []
        while parent is not None and len(chain) < 6:
            chain.append(parent.name)
            parent = parent.cpu_parent
        print(f"{name[:90]:90s} <- {' <- '.join(chain)}")
        n += 1
print("non-in-tree device kernels in one step:", n)
