"""GPU: the bucketed RCCL all-reduce issued from inside the fused backward (with the conv weight
gradients on the aux stream, ops/streams.py) on a 1-rank NCCL(=RCCL) group: every bucket's
collective must be ordered behind both streams, so the reduced (identity) gradients and the updated
parameters equal a run without the reducer."""
import datetime
import socket

import pytest
import torch
import torch.distributed as dist

from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
from proteinbert_pytorch_replication_amd.models import ProteinBERT
from proteinbert_pytorch_replication_amd.parallel.ddp import BucketedAllReduce
from proteinbert_pytorch_replication_amd.train.optim import FusedAdam
from proteinbert_pytorch_replication_amd.train.step import PretrainStep

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(with_ddp: bool, steps: int = 3):
    """Returns the losses, the parameters after ``steps`` updates and the FIRST step's gradients
    (later gradients inherit Adam-amplified float-atomic noise from the diverging parameters)."""
    torch.manual_seed(0)
    m = ProteinBERT(sequences_length=256, num_annotations=512, local_dim=128, global_dim=256, key_dim=64,
                    num_heads=4, num_blocks=3, device="cuda", backend="hip")
    opt = FusedAdam(m.parameters(), lr=1e-3)
    ddp = BucketedAllReduce(opt.arena, bucket_mb=0.5, force=True) if with_ddp else None
    if ddp is not None:
        assert ddp.enabled and len(ddp.buckets) > 4
    step = PretrainStep(m, opt, ddp)
    gen = SyntheticUniRefGO(256, 512, 16, "cuda", seed=5)
    losses, g_first = [], None
    for _ in range(steps):
        X, Y, W = gen.next_batch()
        losses.append(float(step(X, Y, W)))
        if g_first is None:
            g_first = opt.arena.grad.clone()
    torch.cuda.synchronize()
    return losses, opt.arena.data.clone(), g_first


def test_rccl_buckets_behind_aux_stream():
    from proteinbert_pytorch_replication_amd.parallel.dist import nccl_pg_options
    # the process-group options bench.py / pretrain use (high-priority RCCL streams)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                            timeout=datetime.timedelta(seconds=60), device_id=torch.device("cuda", 0),
                            pg_options=nccl_pg_options())
    try:
        l0, p0, g0 = _run(False)
        l1, p1, g1 = _run(True)
    finally:
        dist.destroy_process_group()
    for a, b in zip(l0, l1):
        assert abs(a - b) <= 1e-4 * abs(a) + 1e-6, (l0, l1)
    assert float((g0 - g1).abs().max()) <= 1e-3 * float(g0.abs().max())
    # Adam-normalised updates: see test_graph_step for the bound
    d = (p0 - p1).abs()
    assert float(d.max()) <= 2 * 1e-3 * 3 + 1e-5
    assert float((d > 1e-4).float().mean()) < 0.02



def test_graphed_dp_step_matches_eager_rccl():
    """The whole data-parallel step -- bucket all-reduces launched from the backward's gradient hooks on the
    RCCL communication stream, the overlapped per-bucket Adam, the non-finite checks of the reduced buckets --
    captured once as a hipGraph (train.step.GraphedStep) on a forced 1-rank RCCL group and replayed: same
    losses and parameters over 3 replayed steps as the eager DP step (reference step: utils.py:287-301).
    Runs in its own process (tools/dp_graph_check.py): a failed capture must not take the suite down."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "dp_graph_check.py"), "--port", str(_port())],
                       capture_output=True, text=True, timeout=110, cwd=root)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    out = json.loads(lines[-1])
    assert out["ok"], (out.get("error"), out.get("trace"))
    assert out["buckets"] > 4
    eager, graphed = out["eager"], out["graphed"]
    for a, b in zip(eager[2:], graphed):
        assert abs(a - b) <= 1e-4 * abs(a) + 1e-6, (eager, graphed)
    assert out["steps"] == [5, 5]
    assert out["dmax"] <= 2 * 1e-3 * 3 + 1e-5
    assert out["dfrac"] < 0.02
