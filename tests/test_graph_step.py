"""GPU: the hipGraph-captured training step reproduces the eager step (same data, same updates)."""
import pytest
import torch

from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
from proteinbert_pytorch_replication_amd.models import ProteinBERT
from proteinbert_pytorch_replication_amd.train.optim import FusedAdam
from proteinbert_pytorch_replication_amd.train.step import GraphedStep, PretrainStep

pytestmark = pytest.mark.gpu


def _setup():
    torch.manual_seed(0)
    m = ProteinBERT(sequences_length=128, num_annotations=512, local_dim=128, global_dim=256, key_dim=64,
                    num_heads=4, num_blocks=2, device="cuda", backend="hip")
    opt = FusedAdam(m.parameters(), lr=1e-3)
    gen = SyntheticUniRefGO(128, 512, 8, "cuda", seed=11)
    return m, opt, PretrainStep(m, opt), gen


def test_graphed_step_matches_eager():
    m1, o1, s1, g1 = _setup()
    eager = []
    for _ in range(5):
        X, Y, W = g1.next_batch()
        eager.append(s1(X, Y, W).item())
    m2, o2, s2, g2 = _setup()
    gs = GraphedStep(s2, g2.next_batch, warmup=2)     # consumes steps 1-2
    graphed = [gs().item() for _ in range(3)]          # steps 3-5
    torch.cuda.synchronize()
    for a, b in zip(eager[2:], graphed):
        assert abs(a - b) < 1e-4 * abs(a) + 1e-6, (eager, graphed)
    assert o2.step_count == o1.step_count == 5
    for (n, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        # Adam normalises updates: float-atomic noise in a gradient whose true value is ~0 can flip
        # the sign of an lr-sized step.  Bound every element by the largest possible divergence
        # (2*lr per step after the two shared warmup steps) and require nearly all to agree closely.
        d = (p1 - p2).abs()
        assert float(d.max()) <= 2 * 1e-3 * 3 + 1e-5, n
        assert float((d > 1e-4).float().mean()) < 0.02, (n, float((d > 1e-4).float().mean()))


def test_aux_stream_backward_matches_inline():
    """Conv weight gradients (and the other aux-stream work) on aux streams (ops/streams.py) equal the
    single-stream backward: same kernels, only the streams differ (float-atomic accumulation
    elsewhere in the backward makes the match approximate, not bitwise)."""
    from proteinbert_pytorch_replication_amd.ops import streams
    from proteinbert_pytorch_replication_amd.ops.global_track import unit_loss_grad
    grads = []
    saved = streams.ENABLED
    for enabled in (False, True):
        streams.ENABLED = enabled
        try:
            m, o, s, g = _setup()
            X, Y, W = g.next_batch()
            o.zero_grad()
            loss = s.loss(X, Y, W)
            with unit_loss_grad():
                loss.backward()
            streams.join()
            torch.cuda.synchronize()
            grads.append(o.arena.grad.clone())
        finally:
            streams.ENABLED = saved
    assert torch.isfinite(grads[0]).all()
    scale = float(grads[0].abs().max())
    assert float((grads[0] - grads[1]).abs().max()) <= 1e-3 * scale


def test_prefetched_batches_match_direct():
    """bench.py's side-stream batch producer hands out the same batches, in order, as direct calls."""
    from proteinbert_pytorch_replication_amd.train.step import PrefetchedBatches
    g1 = SyntheticUniRefGO(128, 512, 8, "cuda", seed=5)
    g2 = SyntheticUniRefGO(128, 512, 8, "cuda", seed=5)
    pf = PrefetchedBatches(g2.next_batch, torch.device("cuda"))
    for _ in range(4):
        a, b = g1.next_batch(), pf()
        for da, db in zip(a, b):
            for k in da:
                assert torch.equal(da[k], db[k]), k
