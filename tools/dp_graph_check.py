"""Eager vs hipGraph-captured data-parallel training step on a forced 1-rank RCCL group (one process, one GPU).

Runs 5 eager DP steps and 2 eager + capture + 3 replayed DP steps (train.step.GraphedStep with the bucketed
all-reduce, the overlapped per-bucket Adam and the reduced-gradient non-finite checks), prints one JSON line
with both loss sequences and the parameter difference.  Run as its own process by
tests/test_gpu_ddp_streams.py: a failed capture leaves the RCCL communicator unusable, and tearing that down
aborts the process -- the test suite must survive it.
    python tools/dp_graph_check.py [--port P]
"""
import argparse
import datetime
import json
import os
import sys
import traceback

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO  # noqa: E402
from proteinbert_pytorch_replication_amd.models import ProteinBERT  # noqa: E402
from proteinbert_pytorch_replication_amd.parallel.ddp import BucketedAllReduce  # noqa: E402
from proteinbert_pytorch_replication_amd.parallel.dist import nccl_pg_options  # noqa: E402
from proteinbert_pytorch_replication_amd.train.optim import FusedAdam  # noqa: E402
from proteinbert_pytorch_replication_amd.train.step import GraphedStep, PretrainStep  # noqa: E402


def setup():
    torch.manual_seed(0)
    m = ProteinBERT(sequences_length=256, num_annotations=512, local_dim=128, global_dim=256, key_dim=64,
                    num_heads=4, num_blocks=3, device="cuda", backend="hip")
    opt = FusedAdam(m.parameters(), lr=1e-3)
    ddp = BucketedAllReduce(opt.arena, bucket_mb=0.5, force=True)
    return m, opt, ddp, PretrainStep(m, opt, ddp), SyntheticUniRefGO(256, 512, 16, "cuda", seed=5)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=29531)
    a = ap.parse_args()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{a.port}", rank=0, world_size=1,
                            timeout=datetime.timedelta(seconds=60), device_id=torch.device("cuda", 0),
                            pg_options=nccl_pg_options())
    out = {}
    try:
        _, o1, d1, s1, g1 = setup()
        out["buckets"] = len(d1.buckets)
        out["eager"] = [float(s1(*g1.next_batch())) for _ in range(5)]
        _, o2, _, s2, g2 = setup()
        gs = GraphedStep(s2, g2.next_batch, warmup=2)
        out["graphed"] = [float(gs()) for _ in range(3)]
        torch.cuda.synchronize()
        d = (o1.arena.data - o2.arena.data).abs()
        out["dmax"] = float(d.max())
        out["dfrac"] = float((d > 1e-4).float().mean())
        out["steps"] = [o1.step_count, o2.step_count]
        out["ok"] = True
    except Exception as e:  # noqa: BLE001 - reported to the test
        out["ok"] = False
        out["error"] = f"{type(e).__name__}: {e}"
        out["trace"] = traceback.format_exc()[-3000:]
        print(json.dumps(out), flush=True)
        os._exit(3)            # no process-group teardown after a failed capture (it aborts)
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
