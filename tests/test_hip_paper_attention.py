"""GPU: paper-semantics attention (csrc/paper_attn.hip: split-L masked softmax over positions, fused
tanh/GELU, hand-written backward) against the PyTorch fp32 oracle GlobalAttention.forward_paper
(use_kernel=False): output and gradients w.r.t. h, g, Wq, Wk, Wv, over lengths that give one, several
and ragged L chunks, with padded rows (one row keeps a single valid position)."""
import pytest
import torch

from proteinbert_pytorch_replication_amd.models import ProteinBERT
from proteinbert_pytorch_replication_amd.models.proteinbert import GlobalAttention

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("B,L", [(3, 37), (8, 300), (64, 512), (5, 1000), (600, 128)])
def test_paper_attention_matches_torch(B, L):
    torch.manual_seed(B * 1000 + L)
    H, C, G, K = 4, 128, 512, 64
    att = GlobalAttention(H, C, G, G // H, K, device="cuda", semantics="paper")
    h = (0.3 * torch.randn(B, L, C, device="cuda")).to(torch.bfloat16)
    g = torch.randn(B, G, device="cuda")
    lengths = torch.randint(1, L + 1, (B,), device="cuda")
    lengths[0] = 1
    lengths[-1] = L
    mask = torch.arange(L, device="cuda")[None, :] < lengths[:, None]

    hk = h.clone().requires_grad_(True)
    gk = g.clone().requires_grad_(True)
    out = att.forward_paper(hk, gk, mask)
    dO = torch.randn_like(out)
    (out * dO).sum().backward()
    got = {"o": out.detach(), "h": hk.grad.float(), "g": gk.grad, "Wq": att.Wq.grad.clone(),
           "Wk": att.Wk.grad.clone(), "Wv": att.Wv.grad.clone()}
    att.zero_grad(set_to_none=True)

    hr = h.float().requires_grad_(True)
    gr = g.clone().requires_grad_(True)
    ref_out = att.forward_paper(hr, gr, mask, use_kernel=False)
    (ref_out * dO).sum().backward()
    ref = {"o": ref_out.detach(), "h": hr.grad, "g": gr.grad, "Wq": att.Wq.grad, "Wk": att.Wk.grad,
           "Wv": att.Wv.grad}
    torch.cuda.synchronize()
    for k in ref:
        assert torch.isfinite(got[k]).all(), k
        assert _rel(got[k], ref[k]) < 3e-2, (k, _rel(got[k], ref[k]))
    # padded positions get exactly zero input gradient
    assert (got["h"][~mask] == 0).all()


def test_paper_model_step_uses_kernel_and_matches_oracle():
    from proteinbert_pytorch_replication_amd.ops import paper_attention as pa
    from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
    from proteinbert_pytorch_replication_amd.train.optim import FusedAdam
    from proteinbert_pytorch_replication_amd.train.step import PretrainStep
    torch.manual_seed(0)
    m = ProteinBERT(sequences_length=128, num_annotations=512, local_dim=128, global_dim=512, key_dim=64,
                    num_heads=4, num_blocks=2, device="cuda", semantics="paper")
    X, Y, W = SyntheticUniRefGO(128, 512, 16, "cuda", seed=0).next_batch()
    step = PretrainStep(m, FusedAdam(m.parameters(), lr=2e-4))
    with torch.no_grad():
        pa.ENABLED = False
        try:
            ref = step.loss(X, Y, W).item()
        finally:
            pa.ENABLED = True
        got = step.loss(X, Y, W).item()
    assert abs(got - ref) < 1e-2 * abs(ref), (got, ref)
    losses = [step(X, Y, W).item() for _ in range(5)]
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < losses[0]


@pytest.mark.parametrize("M,K,N", [(1024, 512, 256), (7, 512, 256), (512, 6, 256)])
def test_query_products_fp32_accurate(M, K, N):
    """the paper-semantics query products q = tanh(g Wq), dg = dqpre Wq^T and dWq = g^T dqpre run
    as three-term bf16 hi/lo GEMMs (ops/paper_track.py mm_x3), so their error vs fp64 stays at fp32 level
    (~1e-5 relative) instead of bf16's ~4e-3."""
    from proteinbert_pytorch_replication_amd.ops.global_track import mm32
    from proteinbert_pytorch_replication_amd.ops.paper_track import mm_x3
    torch.manual_seed(M + K)
    a = torch.randn(M, K, device="cuda")
    b = torch.randn(K, N, device="cuda") * 0.05
    ref = a.double() @ b.double()
    err3 = ((mm_x3(a, b).double() - ref).norm() / ref.norm()).item()
    err1 = ((mm32(a.bfloat16(), b.bfloat16()).double() - ref).norm() / ref.norm()).item()
    print(f"M={M} K={K} N={N}: hi/lo rel err {err3:.2e}  plain bf16 {err1:.2e}")
    assert err3 < 2e-5 and err3 < 0.02 * err1
    # non-contiguous operands, as the backward passes them (g^T, Wq^T)
    ref_t = b.t().double() @ a.t().double()
    assert ((mm_x3(b.t(), a.t()).double() - ref_t).norm() / ref_t.norm()).item() < 2e-5
