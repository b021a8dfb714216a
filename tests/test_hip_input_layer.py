"""GPU: the GO-annotation input layer (reference modules.py:255-262,301: g0 = GELU(X W^T + b) and
block 0's global->local vector GELU(g0 Wgl^T + bgl)) in its sparse form (csrc/annot.hip: ordered
CSR/CSC compaction, W^T row gathers, fused bias/GELU and dU/bias/weight-gradient kernels) and its dense
MFMA-GEMM form, against plain PyTorch fp32 at the real width A = 8943: outputs, the weight and bias
gradients, run-to-run bitwise equality of the sparse form, and inputs that are not {0, 1} multi-hot
(values 2, negative values, a fully dense row, blank rows)."""
import pytest
import torch
import torch.nn.functional as F

from proteinbert_pytorch_replication_amd.ops import global_track
from proteinbert_pytorch_replication_amd.ops.global_track import InputLayerFn

pytestmark = pytest.mark.gpu


def _ann(B, A, dev, density=0.005, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = (torch.rand((B, A), device=dev, generator=g) < density).float()
    x[::2] = 0.0                                             # blank rows (the corruption blanks ~half)
    x[1, :7] = 2.0                                           # corruption can add onto a set bit
    if B > 3:
        x[3] = torch.randn(A, device=dev, generator=g)      # a dense, signed row
    return x


def _params(A, G, NGL, dev):
    torch.manual_seed(5)
    w = (torch.randn(G, A, device=dev) * 0.05).requires_grad_()
    b = (torch.randn(G, device=dev) * 0.1).requires_grad_()
    wgl = (torch.randn(NGL, G, device=dev) * G ** -0.5).requires_grad_()
    bgl = (torch.randn(NGL, device=dev) * 0.1).requires_grad_()
    return [w, b, wgl, bgl]


def _run(x, params, dg, dgb):
    for p in params:
        p.grad = None
    g, _g_bf, gb = InputLayerFn.apply(x, *params)
    ((g * dg).sum() + (gb * dgb).sum()).backward()
    torch.cuda.synchronize()
    return g.detach(), gb.detach(), [p.grad.clone() for p in params]


def _relerr(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("sparse", [True, False])
@pytest.mark.parametrize("B,A,G,NGL", [(512, 8943, 512, 128), (37, 8943, 512, 128), (64, 300, 256, 128)])
def test_input_layer_vs_fp32(B, A, G, NGL, sparse, monkeypatch):
    monkeypatch.setattr(global_track, "ANN_SPARSE", sparse)
    dev = torch.device("cuda")
    x = _ann(B, A, dev)
    params = _params(A, G, NGL, dev)
    torch.manual_seed(9)
    dg = torch.randn(B, G, device=dev)
    dgb = torch.randn(B, NGL, device=dev)
    g, gb, grads = _run(x, params, dg, dgb)
    # fp32 reference
    ref = [p.detach().clone().requires_grad_() for p in params]
    g_r = F.gelu(x @ ref[0].t() + ref[1])
    gb_r = F.gelu(g_r @ ref[2].t() + ref[3])
    ((g_r * dg).sum() + (gb_r * dgb).sum()).backward()
    # sparse: fp32 accumulation over bf16 W^T -> ~bf16 rounding of W; dense: bf16 GEMM operands
    assert _relerr(g, g_r.detach()) < 6e-3
    assert _relerr(gb, gb_r.detach()) < 1e-2
    for got, p in zip(grads, ref):
        assert _relerr(got, p.grad) < 1.5e-2, p.shape
    # the weight gradient is exactly zero in every column no annotated row touches
    untouched = (x != 0).sum(0) == 0
    assert torch.all(grads[0][:, untouched] == 0)


def test_input_layer_sparse_deterministic(monkeypatch):
    monkeypatch.setattr(global_track, "ANN_SPARSE", True)
    dev = torch.device("cuda")
    B, A, G, NGL = 512, 8943, 512, 128
    x = _ann(B, A, dev, seed=2)
    params = _params(A, G, NGL, dev)
    dg = torch.randn(B, G, device=dev)
    dgb = torch.randn(B, NGL, device=dev)
    g1, gb1, gr1 = _run(x, params, dg, dgb)
    g2, gb2, gr2 = _run(x, params, dg, dgb)
    assert torch.equal(g1, g2) and torch.equal(gb1, gb2)
    for a, b in zip(gr1[:2], gr2[:2]):
        assert torch.equal(a, b)


def test_input_layer_sparse_matches_dense(monkeypatch):
    """The two forms agree on the GO-shaped input (same bf16 W image precision)."""
    dev = torch.device("cuda")
    B, A, G, NGL = 256, 8943, 512, 128
    x = (torch.rand((B, A), device=dev) < 0.005).float()
    params = _params(A, G, NGL, dev)
    dg = torch.randn(B, G, device=dev)
    dgb = torch.randn(B, NGL, device=dev)
    monkeypatch.setattr(global_track, "ANN_SPARSE", True)
    gs, _, grs = _run(x, params, dg, dgb)
    monkeypatch.setattr(global_track, "ANN_SPARSE", False)
    gd, _, grd = _run(x, params, dg, dgb)
    assert _relerr(gs, gd) < 2e-3
    assert _relerr(grs[0], grd[0]) < 1e-2


def test_input_layer_inference_matches_training_forward(monkeypatch):
    """No-grad forwards build no column lists and run on the current stream only; same outputs."""
    monkeypatch.setattr(global_track, "ANN_SPARSE", True)
    dev = torch.device("cuda")
    B, A, G, NGL = 128, 8943, 512, 128
    x = _ann(B, A, dev, seed=4)
    params = _params(A, G, NGL, dev)
    g_t, _, gb_t = InputLayerFn.apply(x, *params)
    with torch.no_grad():
        g_i, _, gb_i = InputLayerFn.apply(x, *params)
    torch.cuda.synchronize()
    assert torch.equal(g_t.detach(), g_i) and torch.equal(gb_t.detach(), gb_i)
