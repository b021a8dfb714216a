"""GPU: the one-launch fused global-track kernels (csrc/glob2.hip) against the library-GEMM path
(GlobalBlockFn, itself checked against the fp32 reference model in test_hip_local_track): forward
outputs, the input / attention-partial gradients and every parameter gradient."""
import pytest
import torch

from proteinbert_pytorch_replication_amd.ops.global_track import FusedGlobalBlockFn, GlobalBlockFn

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


@pytest.mark.parametrize("B,G,NGL,TV", [(256, 512, 128, 8), (20, 512, 128, 2), (37, 256, 0, 4), (16, 256, 128, 1)])
def test_fused_global_block_matches_library_path(B, G, NGL, TV):
    dev = torch.device("cuda")
    K = 64
    params = _params(G, NGL, K, dev)
    torch.manual_seed(5)
    g0 = torch.randn(B, G, device=dev)
    vp0 = torch.randn(B, TV, G, device=dev) * 0.05
    dg2 = torch.randn(B, G, device=dev)
    dgb = torch.randn(B, NGL, device=dev) if NGL else None
    outs, grads = [], []
    for fn in (GlobalBlockFn, FusedGlobalBlockFn):
        for p in params:
            if p is not None:
                p.grad = None
        g = g0.clone().requires_grad_()
        vp = vp0.clone().requires_grad_()
        g2, g2_bf, gb = fn.apply(g, g.detach().to(torch.bfloat16), vp, *params)
        loss = (g2 * dg2).sum() + ((gb * dgb).sum() if NGL else 0.0)
        loss.backward()
        torch.cuda.synchronize()
        outs.append([g2.detach(), g2_bf.float(), gb.detach()])
        grads.append([g.grad, vp.grad] + [None if p is None else p.grad.clone() for p in params])
    for a, b in zip(*outs):
        if a.numel():
            assert float((a - b).abs().max()) <= 2e-2 * float(a.abs().max()) + 1e-4
    names = ["g", "vpart", "w1", "b1", "n1w", "n1b", "w2", "b2", "n2w", "n2b", "wp", "wgl", "bgl"]
    for n, a, b in zip(names, *grads):
        if a is None:
            assert b is None, n
            continue
        err = float((a - b).abs().max())
        assert err <= 3e-2 * float(a.abs().max()) + 1e-5, (n, err, float(a.abs().max()))
