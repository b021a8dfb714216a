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


@pytest.mark.parametrize("B,G,H,Kd", [(1024, 512, 4, 64), (7, 512, 4, 64), (130, 384, 2, 64), (33, 40, 3, 24)])
def test_query_products_fp32(B, G, H, Kd):
    """the paper-semantics query products q = tanh(g Wq), dg = dqpre Wq^T and dWq += g^T dqpre
    (csrc/sgemm.hip: fp32 FMA, fixed-order split-K, Wq read in place as [H, G, Kd], dqpre = dqs (1 - q^2) /
    sqrt(Kd) formed while staging) stay at fp32 accuracy against fp64 -- bf16 operands would give ~4e-3."""
    from proteinbert_pytorch_replication_amd.ops import _lib
    from proteinbert_pytorch_replication_amd.ops import paper_track  # noqa: F401  (registers the launchers)
    torch.manual_seed(B + G)
    dev = torch.device("cuda")
    st = _lib.stream_ptr(dev)
    g = torch.randn(B, G, device=dev)
    wq = torch.randn(H, G, Kd, device=dev) * 0.05
    s = 1.0 / Kd ** 0.5
    q = torch.empty(B, H * Kd, device=dev)
    qs = torch.empty(B, H * Kd, device=dev)
    ws = torch.empty(_lib.lib().pbx_sg_query_ws(B, G, H, Kd), device=dev)
    _lib.call("pbx_sg_query_fwd", g.data_ptr(), wq.data_ptr(), q.data_ptr(), qs.data_ptr(), ws.data_ptr(), B, G, H, Kd,
              s, st)
    wcat = wq.double().permute(1, 0, 2).reshape(G, H * Kd)
    q_ref = torch.tanh(g.double() @ wcat)
    dqs = torch.randn(B, H * Kd, device=dev)
    dg = torch.empty(B, G, device=dev)
    _lib.call("pbx_sg_query_dg", dqs.data_ptr(), q.data_ptr(), wq.data_ptr(), dg.data_ptr(), ws.data_ptr(), B, G, H,
              Kd, s, st)
    dwq = torch.randn(H, G, Kd, device=dev)
    dwq0 = dwq.clone()
    _lib.call("pbx_sg_query_dwq", g.data_ptr(), dqs.data_ptr(), q.data_ptr(), dwq.data_ptr(), ws.data_ptr(), B, G, H,
              Kd, s, st)
    torch.cuda.synchronize()
    dqpre = dqs.double() * s * (1 - q.double() ** 2)
    dg_ref = dqpre @ wcat.t()
    dwq_ref = dwq0.double() + (g.double().t() @ dqpre).view(G, H, Kd).permute(1, 0, 2)
    rel = lambda a, b: ((a.double() - b).norm() / b.norm()).item()   # noqa: E731
    e_q, e_qs = rel(q, q_ref), rel(qs, q_ref * s)
    e_dg, e_dw = rel(dg, dg_ref), rel(dwq - dwq0, dwq_ref - dwq0.double())
    print(f"B={B} G={G} H={H} Kd={Kd}: q {e_q:.2e} qs {e_qs:.2e} dg {e_dg:.2e} dWq {e_dw:.2e}")
    assert max(e_q, e_qs, e_dg, e_dw) < 2e-6


def test_kv_weight_image_and_gradient_scatter():
    """csrc/sgemm.hip: the fused attention's K/V weight image (bf16 [H][K + VD][C] from Wk [H][C][K] and
    Wv [H][C][VD]) and the dWk / dWv scatter-add from the [C][H K + H VD] GEMM output, vs torch."""
    from proteinbert_pytorch_replication_amd.ops import _lib
    from proteinbert_pytorch_replication_amd.ops import paper_track  # noqa: F401  (registers the launchers)
    torch.manual_seed(7)
    dev = torch.device("cuda")
    st = _lib.stream_ptr(dev)
    H, C, K, VD = 4, 128, 64, 128
    wk = torch.randn(H, C, K, device=dev)
    wv = torch.randn(H, C, VD, device=dev)
    img = torch.empty(H, K + VD, C, dtype=torch.bfloat16, device=dev)
    _lib.call("pbx_pa_wimg", wk.data_ptr(), wv.data_ptr(), img.data_ptr(), H, C, K, VD, st)
    ref = torch.cat([wk.permute(0, 2, 1), wv.permute(0, 2, 1)], dim=1).to(torch.bfloat16)
    dwcat = torch.randn(C, H * (K + VD), device=dev)
    dwk = torch.randn(H, C, K, device=dev)
    dwv = torch.randn(H, C, VD, device=dev)
    rk = dwk + dwcat[:, :H * K].view(C, H, K).permute(1, 0, 2)
    rv = dwv + dwcat[:, H * K:].view(C, H, VD).permute(1, 0, 2)
    _lib.call("pbx_pa_dwkv_add", dwcat.data_ptr(), dwk.data_ptr(), dwv.data_ptr(), H, C, K, VD, st)
    torch.cuda.synchronize()
    assert torch.equal(img, ref)
    assert torch.equal(dwk, rk) and torch.equal(dwv, rv)
