"""GPU: the persistent software-pipelined conv forward (csrc/conv5.hip, pbx_conv_fwd5x) against conv_fwd3
(csrc/conv2.hip) and an fp32 PyTorch oracle.

conv_fwd5 applies the same roundings in the same order (pre-activation + bias to bf16, the build's GELU core,
((x + GELU(n)) + GELU(w)) + gb without FMA contraction, bf16 outputs), so both GELU' images and s1 must be
BITWISE equal to conv_fwd3's; the LayerNorm (mean, M2) tile partials sum the same stored values in another
order.  Shapes cover partial last tiles (odd L), more tiles than workgroups (several rounds per workgroup, a grid tail), fewer tiles
than CUs, context-parallel halo rows, and the inference form (no GELU' images).
Reference: ProteinBERT/modules.py:124-147,205-212.
"""
import pytest
import torch
import torch.nn.functional as F

from proteinbert_pytorch_replication_amd.ops import _lib
from proteinbert_pytorch_replication_amd.ops import local_track as lt

pytestmark = pytest.mark.gpu


def _launch(name, x, wpn, wpw, bn, bw, gb, store, B, L, xlo=0, xhi=0):
    dev = x.device
    gdn = torch.empty(B, L, 128, dtype=torch.bfloat16, device=dev) if store else None
    gdw = torch.empty_like(gdn) if store else None
    s1 = torch.empty(B, L, 128, dtype=torch.bfloat16, device=dev)
    stats = torch.full((B, (L + 127) // 128, 2), float("nan"), device=dev)
    _lib.call(name, x.data_ptr(), wpn.data_ptr(), wpw.data_ptr(), bn.data_ptr(), bw.data_ptr(), gb.data_ptr(),
              lt._p(gdn), lt._p(gdw), s1.data_ptr(), stats.data_ptr(), B, L, 9, 5, xlo, xhi, _lib.stream_ptr(dev))
    return gdn, gdw, s1, stats


def _same(a, b):
    """GELU' images and s1 bitwise (both kernels keep the GELU products out of FMA contraction)."""
    for n, u, v in zip(("gdn", "gdw", "s1"), a[:3], b[:3]):
        if u is None:
            assert v is None
            continue
        assert torch.equal(u, v), (n, (u.float() - v.float()).abs().max().item(), (u != v).float().mean().item())


@pytest.mark.parametrize("B,L,store", [(3, 512, True), (2, 300, True), (5, 77, True), (1, 128, True),
                                       (600, 512, True), (700, 200, True), (4, 1000, False), (300, 512, False)])
def test_conv_fwd5_equals_conv_fwd3(B, L, store):
    torch.manual_seed(B * 1000 + L)
    dev = torch.device("cuda")
    C = 128
    x = (torch.randn(B, L, C, device=dev) * 0.7).to(torch.bfloat16)
    wn, ww = (torch.randn(C, C, 9, device=dev) * 0.04 for _ in range(2))
    bn, bw = torch.randn(C, device=dev) * 0.1, torch.randn(C, device=dev) * 0.1
    gb = torch.randn(B, C, device=dev) * 0.5
    wpn, _ = lt.pack_conv(wn)
    wpw, _ = lt.pack_conv(ww)
    a = _launch("pbx_conv_fwd3x", x, wpn, wpw, bn, bw, gb, store, B, L)
    b = _launch("pbx_conv_fwd5x", x, wpn, wpw, bn, bw, gb, store, B, L)
    torch.cuda.synchronize()
    _same(a, b)
    assert torch.isfinite(b[3]).all()
    torch.testing.assert_close(b[3], a[3], rtol=2e-5, atol=2e-5 * L * C)
    if B * L <= 4000:   # fp32 oracle of the whole forward on the small shapes
        xt = x.float().transpose(1, 2)
        n = F.conv1d(xt, wn.to(torch.bfloat16).float(), bn, padding="same", dilation=1)
        w = F.conv1d(xt, ww.to(torch.bfloat16).float(), bw, padding="same", dilation=5)
        ref = (x.float() + F.gelu(n.transpose(1, 2)) + F.gelu(w.transpose(1, 2)) + gb[:, None, :])
        err = ((b[2].float() - ref).norm() / ref.norm()).item()
        assert err < 1e-2, err


@pytest.mark.parametrize("B,Ls,H", [(3, 256, 20), (2, 300, 20)])
def test_conv_fwd5_context_parallel_rows(B, Ls, H):
    """x carries H rows of the neighbouring shards around each sample's Ls rows (xlo = xhi = H)."""
    torch.manual_seed(Ls)
    dev = torch.device("cuda")
    C = 128
    x = (torch.randn(B, Ls + 2 * H, C, device=dev) * 0.7).to(torch.bfloat16)
    wn, ww = (torch.randn(C, C, 9, device=dev) * 0.04 for _ in range(2))
    bn, bw = torch.randn(C, device=dev) * 0.1, torch.randn(C, device=dev) * 0.1
    gb = torch.randn(B, C, device=dev) * 0.5
    wpn, _ = lt.pack_conv(wn)
    wpw, _ = lt.pack_conv(ww)
    a = _launch("pbx_conv_fwd3x", x, wpn, wpw, bn, bw, gb, True, B, Ls, H, H)
    b = _launch("pbx_conv_fwd5x", x, wpn, wpw, bn, bw, gb, True, B, Ls, H, H)
    torch.cuda.synchronize()
    _same(a, b)
    torch.testing.assert_close(b[3], a[3], rtol=2e-5, atol=2e-5 * Ls * C)


@pytest.mark.parametrize("B,L", [(6, 256), (600, 512), (3, 202)])
def test_conv_fwd5_deterministic(B, L):
    """Repeated launches on the same inputs give bitwise-identical outputs and LayerNorm partials."""
    torch.manual_seed(7)
    dev = torch.device("cuda")
    C = 128
    x = (torch.randn(B, L, C, device=dev) * 0.7).to(torch.bfloat16)
    wn, ww = (torch.randn(C, C, 9, device=dev) * 0.04 for _ in range(2))
    bn, bw = torch.randn(C, device=dev) * 0.1, torch.randn(C, device=dev) * 0.1
    gb = torch.randn(B, C, device=dev) * 0.5
    wpn, _ = lt.pack_conv(wn)
    wpw, _ = lt.pack_conv(ww)
    first = _launch("pbx_conv_fwd5x", x, wpn, wpw, bn, bw, gb, True, B, L)
    for _ in range(10):
        again = _launch("pbx_conv_fwd5x", x, wpn, wpw, bn, bw, gb, True, B, L)
        torch.cuda.synchronize()
        for u, v in zip(first, again):
            assert torch.equal(u, v)
