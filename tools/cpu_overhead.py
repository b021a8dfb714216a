"""Host-side cost of one eager training step vs its GPU time (is the GPU ever starved?).

    python tools/cpu_overhead.py [--batch 512] [--steps 20] [--dp] [--graph]
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
ap.add_argument("--dp", action="store_true",
                help="attach the bucketed all-reduce (forced on a 1-rank RCCL group): the DP step's hooks")
ap.add_argument("--graph", action="store_true", help="time hipGraph replays (GraphedStep) instead of eager steps")
ap.add_argument("--batch-softmax", action="store_true",
                help="with --dp: the local head's batch softmax shared over the (1-rank) group -- its cost")
ap.add_argument("--dp-variant", default="full", choices=["full", "nocomm", "nooverlap"],
                help="--dp diagnosis: nocomm = hooks and flags but no all-reduce; nooverlap = finish() + "
                     "whole-arena Adam")
a = ap.parse_args()
dev = torch.device("cuda", 0)     # an indexed device: init_process_group(device_id=...) requires one
torch.manual_seed(0)
m = ProteinBERT(sequences_length=512, num_annotations=8943, local_dim=128, global_dim=512, key_dim=64, num_heads=4,
                num_blocks=6, device=dev, backend="hip")
opt = FusedAdam(m.parameters(), lr=2e-4)
ddp = None
if a.dp:
    import datetime
    import torch.distributed as dist
    from proteinbert_pytorch_replication_amd.parallel.ddp import BucketedAllReduce
    from proteinbert_pytorch_replication_amd.parallel.dist import nccl_pg_options
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29517", rank=0, world_size=1,
                            timeout=datetime.timedelta(seconds=60), device_id=dev, pg_options=nccl_pg_options())
    ddp = BucketedAllReduce(opt.arena, force=True)
    if a.batch_softmax:
        from proteinbert_pytorch_replication_amd.parallel import batch_softmax
        batch_softmax.enable(force=True)
    if a.dp_variant == "nocomm":
        class _Done:
            def wait(self):
                pass
        dist.all_reduce = lambda *args, **kw: _Done()     # noqa: E731
    elif a.dp_variant == "nooverlap":
        ddp.overlap_optimizer = False
step = PretrainStep(m, opt, ddp)
gen = SyntheticUniRefGO(512, 8943, a.batch, dev, seed=1)
one = lambda: step(*gen.next_batch())  # noqa: E731
if a.graph:
    from proteinbert_pytorch_replication_amd.train.step import GraphedStep
    one = GraphedStep(step, gen.next_batch, warmup=2)
for _ in range(5):
    one()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.steps):
    one()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
mode = ("graph" if a.graph else "eager") + (f" + DP buckets ({len(ddp.buckets)}, 1-rank RCCL, {a.dp_variant})"
                                            if ddp else "") + (" + shared batch softmax" if a.batch_softmax else "")
print(f"B={a.batch} {mode}: issue {1000 * (t1 - t0) / a.steps:.3f} ms/step   complete {1000 * (t2 - t0) / a.steps:.3f} "
      "ms/step", flush=True)
if os.environ.get("PBX_CPROFILE"):
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        one()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(35)
if ddp is not None:
    import torch.distributed as dist
    dist.destroy_process_group()
