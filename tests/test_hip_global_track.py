"""GPU: the fused global-track kernels -- the column-split forward (csrc/glob3.hip) and the one-launch
backward (csrc/glob2.hip) -- against a plain PyTorch fp32 evaluation of the same block math
(reference modules.py:175-199,219-229, reference semantics): forward outputs, the input / attention-
partial gradients and every parameter gradient.  The kernels use bf16 GEMM operands (activations and
weight mirrors), so the tolerances are bf16-level relative errors."""
import pytest
import torch
import torch.nn.functional as F

from proteinbert_pytorch_replication_amd.ops import global_track
from proteinbert_pytorch_replication_amd.ops.global_track import FusedGlobalBlockFn

pytestmark = pytest.mark.gpu


def _params(G, NGL, K, dev):
    torch.manual_seed(3)
    mk = lambda *s, sc=1.0: (torch.randn(*s, device=dev) * sc).requires_grad_()  # noqa: E731
    p = [mk(G, G, sc=G ** -0.5), mk(G, sc=0.1), (1 + 0.1 * torch.randn(G, device=dev)).requires_grad_(),
         mk(G, sc=0.1), mk(G, G, sc=G ** -0.5), mk(G, sc=0.1), (1 + 0.1 * torch.randn(G, device=dev)).requires_grad_(),
         mk(G, sc=0.1), mk(K, sc=1.0)]
    if NGL:
        p += [mk(NGL, G, sc=G ** -0.5), mk(NGL, sc=0.1)]
    else:
        p += [None, None]
    return p


def _reference(g, vp, w1, b1, n1w, n1b, w2, b2, n2w, n2b, wp, wgl, bgl):
    """fp32 torch: g1 = LN(g + GELU(g W1^T + b1) + mean(wp) sum_t vp), g2 = LN(g1 + GELU(g1 W2^T + b2)),
    gb = GELU(g2 Wgl^T + bgl)."""
    G = g.shape[1]
    z1 = g + F.gelu(g @ w1.t() + b1) + wp.mean() * vp.sum(dim=1)
    g1 = F.layer_norm(z1, (G,), n1w, n1b, eps=1e-5)
    g2 = F.layer_norm(g1 + F.gelu(g1 @ w2.t() + b2), (G,), n2w, n2b, eps=1e-5)
    gb = F.gelu(g2 @ wgl.t() + bgl) if wgl is not None else torch.zeros((g.shape[0], 0), device=g.device)
    return g2, gb


def _run(fn_apply, params, g0, vp0, dg2, dgb, NGL):
    for p in params:
        if p is not None:
            p.grad = None
    g = g0.clone().requires_grad_()
    vp = vp0.clone().requires_grad_()
    g2, gb = fn_apply(g, vp)
    loss = (g2 * dg2).sum() + ((gb * dgb).sum() if NGL else 0.0)
    loss.backward()
    torch.cuda.synchronize()
    return [g2.detach(), gb.detach()], [g.grad, vp.grad] + [None if p is None else p.grad.clone() for p in params]


@pytest.mark.parametrize("B,G,NGL,TV", [(512, 512, 128, 8), (256, 512, 128, 8), (20, 512, 128, 2),
                                        (37, 256, 0, 4), (16, 256, 128, 1), (64, 512, 128, 16)])
def test_fused_global_block_vs_fp32(B, G, NGL, TV):
    _check_fused_global_block(B, G, NGL, TV)


def _check_fused_global_block(B, G, NGL, TV):
    dev = torch.device("cuda")
    K = 64
    params = _params(G, NGL, K, dev)
    torch.manual_seed(5)
    g0 = torch.randn(B, G, device=dev)
    vp0 = torch.randn(B, TV, G, device=dev) * 0.05
    dg2 = torch.randn(B, G, device=dev)
    dgb = torch.randn(B, NGL, device=dev) if NGL else None

    def fused(g, vp):
        g2, _, gb = FusedGlobalBlockFn.apply(g, g.detach().to(torch.bfloat16), vp, *params)
        return g2, gb

    out_f, grad_f = _run(fused, params, g0, vp0, dg2, dgb, NGL)
    out_r, grad_r = _run(lambda g, vp: _reference(g, vp, *params), params, g0, vp0, dg2, dgb, NGL)
    for name, a, b in zip(["g2", "gb"], out_r, out_f):
        if a.numel():
            err = float((a - b).abs().max())
            print(f"{name}: max |err| {err:.3e} (max |ref| {float(a.abs().max()):.3e})")
            assert err <= 1.5e-2 * float(a.abs().max()) + 1e-4, (name, err)
    names = ["g", "vpart", "w1", "b1", "n1w", "n1b", "w2", "b2", "n2w", "n2b", "wp", "wgl", "bgl"]
    for n, a, b in zip(names, grad_r, grad_f):
        if a is None:
            assert b is None, n
            continue
        err = float((a - b).abs().max())
        rel = float((a - b).norm() / (a.norm() + 1e-30))
        print(f"d{n}: max |err| {err:.3e} rel-l2 {rel:.2e}")
        assert err <= 2.5e-2 * float(a.abs().max()) + 1e-5, (n, err, float(a.abs().max()))
        assert rel <= 1.2e-2, (n, rel)


@pytest.mark.parametrize("B,G,NGL,TV", [(37, 512, 128, 4), (24, 384, 128, 2), (16, 256, 0, 1)])
def test_general_global_block_vs_fp32(B, G, NGL, TV):
    """The general-shape global track (GlobalBlockFn: in-tree GEMMs + the row LayerNorm kernels of
    csrc/glob.hip), used when the fused kernels do not cover (G, NGL), e.g. G = 384."""
    from proteinbert_pytorch_replication_amd.ops.global_track import GlobalBlockFn
    dev = torch.device("cuda")
    params = _params(G, NGL, 64, dev)
    torch.manual_seed(7)
    g0 = torch.randn(B, G, device=dev)
    vp0 = torch.randn(B, TV, G, device=dev) * 0.05
    dg2 = torch.randn(B, G, device=dev)
    dgb = torch.randn(B, NGL, device=dev) if NGL else None

    def general(g, vp):
        g2, _, gb = GlobalBlockFn.apply(g, g.detach().to(torch.bfloat16), vp, *params)
        return g2, gb

    out_f, grad_f = _run(general, params, g0, vp0, dg2, dgb, NGL)
    out_r, grad_r = _run(lambda g, vp: _reference(g, vp, *params), params, g0, vp0, dg2, dgb, NGL)
    for name, a, b in zip(["g2", "gb"], out_r, out_f):
        if a.numel():
            err = float((a - b).abs().max())
            print(f"{name}: max |err| {err:.3e} (max |ref| {float(a.abs().max()):.3e})")
            assert err <= 1.5e-2 * float(a.abs().max()) + 1e-4, (name, err)
    names = ["g", "vpart", "w1", "b1", "n1w", "n1b", "w2", "b2", "n2w", "n2b", "wp", "wgl", "bgl"]
    for n, a, b in zip(names, grad_r, grad_f):
        if a is None:
            assert b is None, n
            continue
        rel = float((a - b).norm() / (a.norm() + 1e-30))
        print(f"d{n}: rel-l2 {rel:.2e}")
        assert rel <= 1.2e-2, (n, rel)
