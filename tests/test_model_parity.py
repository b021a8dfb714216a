"""Parity of the eager (torch) model against the reference ``modules.py`` (fp32 CPU)."""
import pytest
import torch

from proteinbert_pytorch_replication_amd.models import ProteinBERT
from proteinbert_pytorch_replication_amd.train.losses import pretrain_loss_torch
from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO

CFG = dict(sequences_length=32, num_annotations=40, local_dim=16, global_dim=32, key_dim=8,
           num_heads=4, num_blocks=2)


def _pair(reference_modules, seed=0):
    torch.manual_seed(seed)
    ref = reference_modules.ProteinBERT(device="cpu", **CFG)
    ours = ProteinBERT(backend="torch", **CFG)
    ours.load_state_dict(ref.state_dict(), strict=True)
    for i, blk in enumerate(ref.proteinBERT_blocks):
        heads = blk.global_attention_layer.global_attention_heads
        att = ours.proteinBERT_blocks[i].global_attention_layer
        with torch.no_grad():
            for j, h in enumerate(heads):
                att.Wv[j].copy_(h.Wv_parameter)
                att.Wk[j].copy_(h.Wk_parameter)
                att.Wq[j].copy_(h.Wq_parameter)
    return ref, ours


def _batch(B=3, seed=1):
    gen = SyntheticUniRefGO(CFG["sequences_length"], CFG["num_annotations"], B, "cpu", seed=seed,
                            density=0.1, use_kernel=False)
    return gen.next_batch()


def test_state_dict_keys_match_reference(reference_modules):
    ref, ours = _pair(reference_modules)
    rk, ok = ref.state_dict(), ours.state_dict()
    assert list(rk.keys()) == list(ok.keys())
    for k in rk:
        assert rk[k].shape == ok[k].shape, k


def test_paper_config_has_133_keys():
    m = ProteinBERT(sequences_length=8, num_annotations=8943, local_dim=128, global_dim=512, key_dim=64,
                    num_heads=4, num_blocks=6, backend="torch")
    assert len(m.state_dict()) == 133
    n_reg = sum(p.numel() for p in m.parameters())
    # registered params at L=8: 15,388,809 at L=256 minus the LN(L,C) difference
    assert n_reg == 15_388_809 - 6 * 4 * (256 - 8) * 128


def test_forward_parity(reference_modules):
    ref, ours = _pair(reference_modules)
    X, Y, W = _batch()
    with torch.no_grad():
        pl_r, pg_r = ref(X)
        pl_o, pg_o = ours(X)
    torch.testing.assert_close(pl_o, pl_r, rtol=2e-5, atol=2e-6)
    torch.testing.assert_close(pg_o, pg_r, rtol=2e-5, atol=2e-6)


def test_faithful_attention_equals_closed_form(reference_modules):
    _, ours = _pair(reference_modules)
    X, _, _ = _batch()
    with torch.no_grad():
        a = ours.encode_torch(X["local"], X["global"], faithful_attention=True)
        b = ours.encode_torch(X["local"], X["global"], faithful_attention=False)
    torch.testing.assert_close(a[0], b[0], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(a[1], b[1], rtol=1e-5, atol=1e-5)


def test_loss_and_grad_parity(reference_modules):
    ref, ours = _pair(reference_modules)
    X, Y, W = _batch()
    W64 = {k: v.double() for k, v in W.items()}
    ce, bce = torch.nn.CrossEntropyLoss(reduction="none"), torch.nn.BCELoss(reduction="none")
    pl, pg = ref(X)
    loss_r = torch.mean(ce(pl.permute(0, 2, 1), Y["local"]) * W64["local"]) + \
        torch.mean(bce(pg, Y["global"].float()) * W64["global"])
    loss_r.backward()
    pl, pg = ours(X)
    loss_o = pretrain_loss_torch(pl, pg, Y, W)
    loss_o.backward()
    assert abs(loss_o.item() - loss_r.item()) < 1e-5
    rp = dict(ref.named_parameters())
    for n, p in ours.named_parameters():
        if n.endswith(("Wv", "Wk", "Wq")):
            continue
        g_r, g_o = rp[n].grad, p.grad
        scale = g_r.abs().max().item() + 1e-12
        assert (g_o - g_r).abs().max().item() <= 1e-4 * scale + 1e-7, n


def test_standalone_attention_head_matches_reference(reference_modules):
    """``GlobalAttentionHead`` (reference ``modules.py:21-60``): same parameters, same [B, K, vd] output;
    the closed form equals the literal computation, and in paper semantics every row is the
    position-softmax single-query attention."""
    from proteinbert_pytorch_replication_amd.models import GlobalAttentionHead
    torch.manual_seed(3)
    ref = reference_modules.GlobalAttentionHead(16, 32, 8, 8, device="cpu")
    ours = GlobalAttentionHead(16, 32, 8, 8)
    ours.load_state_dict(ref.state_dict(), strict=True)
    x = {"local": torch.randn(3, 20, 16) * 0.3, "global": torch.randn(3, 32) * 0.3}
    with torch.no_grad():
        r = ref(x)
        torch.testing.assert_close(ours(x), r, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(ours.forward_faithful(x), r, rtol=1e-5, atol=1e-6)
        ours.semantics = "paper"
        o = ours(x)
        q = torch.tanh(x["global"] @ ours.Wq_parameter)
        k = torch.tanh(x["local"] @ ours.Wk_parameter)
        p = torch.softmax((k @ q.unsqueeze(-1)).squeeze(-1) / 8 ** 0.5, dim=-1)
        v = torch.nn.functional.gelu(x["local"] @ ours.Wv_parameter)
        torch.testing.assert_close(o[:, 5], (p.unsqueeze(-1) * v).sum(1), rtol=1e-5, atol=1e-6)
