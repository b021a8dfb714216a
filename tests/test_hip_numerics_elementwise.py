"""GPU numerics, element-wise: the fused first-block / LayerNorm-1 backward paths vs plain PyTorch fp32.

The other kernel tests bound relative Frobenius norms; these bound the per-element error distribution
(normalised max error and a high percentile of the element-wise relative error) at an odd sequence length
(L = 500: partial 128-row conv tiles, partial 32-position pool tiles, odd 2-position LN1 pairs) and B = 1,
for the two round-4 fusions:
  * ``conv_dgrad4<FIN>`` (csrc/conv4.hip, the LayerNorm-1 backward finalize fused into the conv data
    gradient's staging pass) -- checked on dx, dgb and the conv weight gradients of a block;
  * the embedding fold of the first block (csrc/ln.hip ``embed_bwd<true>`` + csrc/wgrad.hip ``wgrad_tok``:
    dE from the token one-hot sums, no conv data gradient) -- checked on the embedding gradient;
and a per-parameter check of the four [L, C] LayerNorm affine gradients with no model-wide slack.
Reference math: ProteinBERT/modules.py:201-219 (block), :249-253 (embedding); reference semantics.
"""
import pytest
import torch

from proteinbert_pytorch_replication_amd.models import ProteinBERT

from test_hip_local_track import make_block, torch_local

pytestmark = pytest.mark.gpu


def elementwise(got, ref, floor=0.1):
    """(max |err| / max |ref|, 99.9th percentile of |err| / (|ref| + floor * rms(ref)))."""
    a, b = got.detach().float().reshape(-1), ref.detach().float().reshape(-1)
    err = (a - b).abs()
    nmax = (err.max() / b.abs().max().clamp_min(1e-30)).item()
    rms = b.pow(2).mean().sqrt().clamp_min(1e-30)
    relv = err / (b.abs() + floor * rms)
    p999 = torch.quantile(relv[torch.randperm(relv.numel(), device=relv.device)[:1 << 20]], 0.999).item()
    return nmax, p999


@pytest.mark.parametrize("fin", [True, False])
@pytest.mark.parametrize("L,B", [(500, 1), (500, 2), (130, 1)])
def test_block_backward_elementwise_vs_fp32(L, B, fin, monkeypatch):
    """One block's backward with (fin) and without the fused LN1 finalize: per-element errors of dx, dgb
    and both conv weight gradients against fp32 autograd of the same block."""
    from proteinbert_pytorch_replication_amd.ops import local_track
    from proteinbert_pytorch_replication_amd.ops.local_track import local_block
    monkeypatch.setattr(local_track, "DGRAD_FIN", fin)
    m, blk = make_block(L, seed=11)
    torch.manual_seed(L * 7 + B)
    x0 = torch.randn(B, L, 128, device="cuda").to(torch.bfloat16)
    gb0 = torch.randn(B, 128, device="cuda") * 0.5
    dh = torch.randn(B, L, 128, device="cuda")
    dv = torch.randn(B, 512, device="cuda") * 1e-2
    wn, ww = blk.local_narrow_conv_layer[0].weight, blk.local_wide_conv_layer[0].weight
    x = x0.clone().requires_grad_(True)
    gb = gb0.clone().requires_grad_(True)
    h2, vpart = local_block(x, gb, blk)
    got = torch.autograd.grad((h2.float() * dh).sum() + (vpart.sum(1) * dv).sum(), [x, gb, wn, ww])
    xr = x0.float().clone().requires_grad_(True)
    gbr = gb0.clone().requires_grad_(True)
    rh2, rv = torch_local(xr, gbr, blk)
    ref = torch.autograd.grad((rh2 * dh).sum() + (rv * dv).sum(), [xr, gbr, wn, ww])
    torch.cuda.synchronize()
    # bounds ~2x the MI355X observations (max over the cases, round 5): dx 8.2e-3 / 7.1e-2, dgb 2.6e-3 /
    # 5.5e-2, dWn / dWw 5.5e-3 / 8.8e-2 -- bf16 dx and bf16 intermediates (s1, h1, s2, h2, dh2, dS1, dpre)
    bounds = {"dx": (1.6e-2, 0.15), "dgb": (6e-3, 0.12), "dWn": (1.2e-2, 0.18), "dWw": (1.2e-2, 0.18)}
    for name, a, b in zip(bounds, got, ref):
        nmax, p999 = elementwise(a, b)
        print(f"L={L} B={B} fin={fin} {name}: max|err|/max|ref| {nmax:.2e}  p99.9 rel {p999:.2e}")
        assert nmax < bounds[name][0] and p999 < bounds[name][1], (name, nmax, p999)


@pytest.mark.parametrize("L,B", [(500, 1), (500, 3)])
def test_embedding_fold_elementwise_vs_fp32(L, B):
    """First-block embedding fold (dE = sum_tok (dS1 + conv^T dpre) from the token one-hot sums, no conv
    data gradient) vs fp32 autograd of the same 1-block model: per-element errors of the embedding
    gradient and the first block's conv weight gradients (the one-hot wgrad_tok path)."""
    from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
    from proteinbert_pytorch_replication_amd.ops.fused_model import fused_pretrain_loss
    from proteinbert_pytorch_replication_amd.train.losses import pretrain_loss_torch
    torch.manual_seed(1)
    A = 512
    m = ProteinBERT(sequences_length=L, num_annotations=A, local_dim=128, global_dim=512, key_dim=64, num_heads=4,
                    num_blocks=1, device="cuda", backend="hip")
    X, Y, W = SyntheticUniRefGO(L, A, B, "cuda", seed=4).next_batch()
    fused_pretrain_loss(m, X, Y, W).backward()
    from proteinbert_pytorch_replication_amd.ops import streams
    streams.join()
    names = ["local_embedding.weight", "proteinBERT_blocks.0.local_narrow_conv_layer.0.weight",
             "proteinBERT_blocks.0.local_wide_conv_layer.0.weight"]
    params = dict(m.named_parameters())
    got = {n: params[n].grad.detach().clone() for n in names}
    m.zero_grad(set_to_none=True)
    h, g = m.encode_torch(X["local"], X["global"], torch.float32)
    pl, pg = m.heads_torch(h, g)
    pretrain_loss_torch(pl, pg, Y, {k: v.float() for k, v in W.items()}).backward()
    torch.cuda.synchronize()
    for n in names:
        ref = params[n].grad
        used = ref.abs().sum(dim=tuple(range(1, ref.dim()))) > 0      # tokens absent from the batch: exact 0
        nmax, p999 = elementwise(got[n][used], ref[used])
        print(f"L={L} B={B} {n}: max|err|/max|ref| {nmax:.2e}  p99.9 rel {p999:.2e}")
        # observed (round 5): max 1.0e-2 / p99.9 0.18 (the embedding: its 26 rows sum ~19 K positions each)
        assert nmax < 2e-2 and p999 < 0.25, (n, nmax, p999)
        assert torch.count_nonzero(got[n][~used]) == 0


@pytest.mark.parametrize("L,nblocks", [(500, 2), (256, 1)])
def test_layernorm_affine_grads_per_parameter(L, nblocks):
    """The [L, C] LayerNorm affine gradients of every block, each against its own fp32 reference: relative
    norm per parameter and per position row (99th percentile over rows) -- no model-wide slack term."""
    from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
    from proteinbert_pytorch_replication_amd.ops.fused_model import fused_pretrain_loss
    from proteinbert_pytorch_replication_amd.train.losses import pretrain_loss_torch
    torch.manual_seed(2)
    A = 512
    m = ProteinBERT(sequences_length=L, num_annotations=A, local_dim=128, global_dim=512, key_dim=64, num_heads=4,
                    num_blocks=nblocks, device="cuda", backend="hip")
    with torch.no_grad():
        for blk in m.proteinBERT_blocks:
            for ln in (blk.local_norm_1, blk.local_norm_2):
                ln.weight.normal_(1.0, 0.2)
                ln.bias.normal_(0.0, 0.2)
    X, Y, W = SyntheticUniRefGO(L, A, 4, "cuda", seed=6).next_batch()
    fused_pretrain_loss(m, X, Y, W).backward()
    from proteinbert_pytorch_replication_amd.ops import streams
    streams.join()
    names = [n for n, p in m.named_parameters() if "local_norm" in n]
    params = dict(m.named_parameters())
    got = {n: params[n].grad.detach().clone() for n in names}
    m.zero_grad(set_to_none=True)
    h, g = m.encode_torch(X["local"], X["global"], torch.float32)
    pl, pg = m.heads_torch(h, g)
    pretrain_loss_torch(pl, pg, Y, {k: v.float() for k, v in W.items()}).backward()
    torch.cuda.synchronize()
    assert len(names) == 4 * nblocks
    for n in names:
        a, b = got[n].float(), params[n].grad.float()
        assert a.shape == (L, 128)
        whole = ((a - b).norm() / b.norm()).item()
        rows = ((a - b).norm(dim=1) / b.norm(dim=1).clamp_min(1e-3 * b.norm(dim=1).mean())).quantile(0.99).item()
        print(f"{n:50s} rel {whole:.2e}  rows p99 {rows:.2e}")
        # observed (round 5): rel <= 9.7e-3, rows p99 <= 1.45e-2
        assert whole < 2e-2 and rows < 3e-2, (n, whole, rows)
