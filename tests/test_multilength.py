"""Multi-length training: the reference's LayerNorm((L, C)) affine ties a model to one L
(modules.py:148-151; any other L raises).  ProteinBERT(variable_length=True) stores the affine at
L_max and slices it per batch; a batch at L must reproduce a fixed-L model holding the first L rows."""
import pytest
import torch

from proteinbert_pytorch_replication_amd.data import MultiLengthSynthetic, SyntheticUniRefGO
from proteinbert_pytorch_replication_amd.models import ProteinBERT
from proteinbert_pytorch_replication_amd.train.losses import pretrain_loss_torch
from proteinbert_pytorch_replication_amd.train.optim import FusedAdam
from proteinbert_pytorch_replication_amd.train.step import PretrainStep

CFG = dict(num_annotations=40, local_dim=16, global_dim=32, key_dim=8, num_heads=4, num_blocks=2)


def _loss(m, batch):
    X, Y, W = batch
    h, g = m.encode_torch(X["local"], X["global"], torch.float32)
    pl, pg = m.heads_torch(h, g)
    return pretrain_loss_torch(pl, pg, Y, {k: v.float() for k, v in W.items()})


def test_sliced_affine_equals_fixed_length_model():
    torch.manual_seed(0)
    big = ProteinBERT(sequences_length=64, variable_length=True, backend="torch", **CFG)
    with torch.no_grad():
        for blk in big.proteinBERT_blocks:
            for ln in (blk.local_norm_1, blk.local_norm_2):
                ln.weight.normal_(1.0, 0.3)
                ln.bias.normal_(0.0, 0.3)
    small = ProteinBERT(sequences_length=24, backend="torch", **CFG)
    sd = {k: (v[:24] if "local_norm" in k else v) for k, v in big.state_dict().items()}
    small.load_state_dict(sd)
    small.load_attention_heads_state(big.attention_heads_state())
    batch = SyntheticUniRefGO(24, 40, 3, "cpu", seed=1, use_kernel=False).next_batch()
    lb, ls = _loss(big, batch), _loss(small, batch)
    assert torch.allclose(lb, ls, rtol=1e-6, atol=1e-7)
    lb.backward()
    ls.backward()
    for (n, pb), (_, ps) in zip(big.named_parameters(), small.named_parameters()):
        if "local_norm" in n:
            assert torch.allclose(pb.grad[:24], ps.grad, rtol=1e-5, atol=1e-7), n
            assert float(pb.grad[24:].abs().max()) == 0.0, n          # rows beyond L get no gradient
        else:
            assert torch.allclose(pb.grad, ps.grad, rtol=1e-5, atol=1e-7), n


def test_fixed_length_model_rejects_other_lengths():
    m = ProteinBERT(sequences_length=32, backend="torch", **CFG)
    batch = SyntheticUniRefGO(16, 40, 2, "cpu", seed=1, use_kernel=False).next_batch()
    with pytest.raises(RuntimeError, match="variable_length"):
        _loss(m, batch)
    v = ProteinBERT(sequences_length=32, variable_length=True, backend="torch", **CFG)
    long_batch = SyntheticUniRefGO(48, 40, 2, "cpu", seed=1, use_kernel=False).next_batch()
    with pytest.raises(RuntimeError):
        _loss(v, long_batch)                                             # L > L_max


def test_multilength_schedule_trains():
    torch.manual_seed(0)
    m = ProteinBERT(sequences_length=64, variable_length=True, backend="torch", **CFG)
    opt = FusedAdam(m.parameters(), lr=1e-3)
    step = PretrainStep(m, opt)
    gen = MultiLengthSynthetic((16, 32, 64), 40, 4, "cpu", use_kernel=False)
    seen = []
    for _ in range(6):
        X, Y, W = gen.next_batch()
        seen.append(X["local"].shape[1])
        assert torch.isfinite(step(X, Y, W))
    assert seen == [16, 32, 64, 16, 32, 64]


@pytest.mark.gpu
def test_hip_variable_length_matches_torch():
    """HIP executor at L < L_max: the kernels read the first L rows of the [L_max, C] affine and
    accumulate its gradient there."""
    from proteinbert_pytorch_replication_amd.ops.fused_model import fused_pretrain_loss
    torch.manual_seed(0)
    m = ProteinBERT(sequences_length=512, num_annotations=8943, local_dim=128, global_dim=512, key_dim=64,
                    num_heads=4, num_blocks=2, device="cuda", backend="hip", variable_length=True)
    batch = SyntheticUniRefGO(200, 8943, 8, "cuda", seed=3).next_batch()
    loss = fused_pretrain_loss(m, *batch)
    loss.backward()
    got = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    m.zero_grad(set_to_none=True)
    lref = _loss(m, batch)
    lref.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - lref.item()) < 2e-3 * abs(lref.item())
    for n, p in m.named_parameters():
        if "local_norm" in n:
            assert float(got[n][200:].abs().max()) == 0.0, n
            err = (got[n][:200] - p.grad[:200]).norm().item()
            assert err < 3e-2 * p.grad[:200].norm().item() + 1e-6, n


def test_variable_length_model_roundtrips_through_checkpoint(tmp_path):
    """variable_length is part of model.config: a multi-length model saved with save_final_model
    reloads as a multi-length model that still accepts L < L_max."""
    from proteinbert_pytorch_replication_amd.train.checkpoint import load_model, save_final_model
    torch.manual_seed(0)
    m = ProteinBERT(sequences_length=48, variable_length=True, backend="torch", **CFG)
    path = save_final_model(m, str(tmp_path))
    r = load_model(path, device="cpu", backend="torch")
    assert r.variable_length and r.config["variable_length"]
    batch = SyntheticUniRefGO(20, 40, 2, "cpu", seed=2, use_kernel=False).next_batch()
    assert torch.allclose(_loss(m, batch), _loss(r, batch), rtol=1e-6, atol=1e-7)
