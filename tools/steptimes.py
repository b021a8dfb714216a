"""Per-step wall times of the headline training step (variance study): prints min / median / max ms."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from proteinbert_pytorch_replication_amd.config import get_preset  # noqa: E402
from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO  # noqa: E402
from proteinbert_pytorch_replication_amd.models import ProteinBERT  # noqa: E402
from proteinbert_pytorch_replication_amd.train.optim import FusedAdam  # noqa: E402
from proteinbert_pytorch_replication_amd.train.step import PretrainStep  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
cfg = get_preset("cfg2_paper_l512").model
dev = torch.device("cuda")
torch.manual_seed(0)
m = ProteinBERT(sequences_length=512, num_annotations=cfg.num_annotations, local_dim=128, global_dim=512, key_dim=64,
                num_heads=4, num_blocks=6, device=dev, backend="hip")
opt = FusedAdam(m.parameters(), lr=2e-4)
step = PretrainStep(m, opt)
gen = SyntheticUniRefGO(512, cfg.num_annotations, 256, dev, seed=1)
for _ in range(5):
    step(*gen.next_batch())
torch.cuda.synchronize()
ts = []
for _ in range(steps):
    t0 = time.perf_counter()
    step(*gen.next_batch())
    torch.cuda.synchronize()
    ts.append(1000 * (time.perf_counter() - t0))
ts.sort()
print(f"per-step ms (synchronised each step): min {ts[0]:.3f} p25 {ts[len(ts)//4]:.3f} median {ts[len(ts)//2]:.3f} "
      f"p75 {ts[3*len(ts)//4]:.3f} max {ts[-1]:.3f}", flush=True)
