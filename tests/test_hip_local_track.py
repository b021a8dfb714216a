"""GPU numerics: fused CDNA4 local-track kernels vs a plain PyTorch fp32 reference of the same math.

The reference math is ProteinBERT/modules.py:201-219 (reference semantics: LayerNorm over (L, C),
attention reduced to (1/K) sum_l GELU(h Wv)).  Odd sequence lengths exercise the
partial tiles and the zero-padded conv halo at sequence ends.
"""
import pytest
import torch
import torch.nn.functional as F

from proteinbert_pytorch_replication_amd.models import ProteinBERT

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def make_block(L, G=512, seed=0):
    torch.manual_seed(seed)
    m = ProteinBERT(sequences_length=L, num_annotations=64, local_dim=128, global_dim=G, key_dim=64, num_heads=4,
                    num_blocks=1, device="cuda", backend="hip")
    blk = m.proteinBERT_blocks[0]
    with torch.no_grad():  # non-trivial affine params
        for ln in (blk.local_norm_1, blk.local_norm_2):
            ln.weight.normal_(1.0, 0.2)
            ln.bias.normal_(0.0, 0.2)
    return m, blk


def torch_local(x, gb, blk):
    """fp32 reference of the fused local track: returns (h2, vsum)."""
    nc, wc = blk.local_narrow_conv_layer[0], blk.local_wide_conv_layer[0]
    xt = x.transpose(1, 2)
    n = F.gelu(F.conv1d(xt, nc.weight, nc.bias, padding="same", dilation=1)).transpose(1, 2)
    w = F.gelu(F.conv1d(xt, wc.weight, wc.bias, padding="same", dilation=blk.wide_conv_dilation)).transpose(1, 2)
    s1 = x + n + w + gb.unsqueeze(1)
    h1 = F.layer_norm(s1, blk.local_norm_1.normalized_shape, blk.local_norm_1.weight, blk.local_norm_1.bias)
    lin = blk.local_linear_layer[0]
    s2 = h1 + F.gelu(F.linear(h1, lin.weight, lin.bias))
    h2 = F.layer_norm(s2, blk.local_norm_2.normalized_shape, blk.local_norm_2.weight, blk.local_norm_2.bias)
    wv = blk.global_attention_layer.value_weight_cat()
    vsum = F.gelu(h2 @ wv).sum(dim=1)
    return h2, vsum


@pytest.mark.parametrize("L,B,frozen", [(512, 3, False), (200, 2, False), (300, 2, False), (64, 4, False),
                                        (1024, 2, False), (4096, 1, False), (512, 3, True), (300, 2, True),
                                        (4096, 1, True)])
def test_local_block_forward(L, B, frozen):
    """frozen: no input needs a gradient (frozen-encoder / inference forward): no backward state (conv
    GELU' images, MLP pre-activation) is written."""
    from proteinbert_pytorch_replication_amd.ops.local_track import local_block
    m, blk = make_block(L)
    if frozen:
        blk.requires_grad_(False)
    x = torch.randn(B, L, 128, device="cuda").to(torch.bfloat16)
    gb = torch.randn(B, 128, device="cuda") * 0.5
    with torch.no_grad():
        h2, vpart = local_block(x, gb, blk)
        rh2, rv = torch_local(x.float(), gb, blk)
    torch.cuda.synchronize()
    e_h, e_v = rel(h2, rh2), rel(vpart.sum(1), rv)
    print(f"L={L} B={B} frozen={frozen}: rel h2 {e_h:.2e} vsum {e_v:.2e}")
    assert e_h < 1.5e-2
    assert e_v < 1.5e-2


# conv: 3 = conv_fwd3 + conv_dgrad4 with the LN1 finalize fused in (default), 5 = the same with a separate
# ln1_finalize; the pool is csrc/pool.hip (GELU' recomputed in the backward)
@pytest.mark.parametrize("conv", [3, 5])
@pytest.mark.parametrize("L,B", [(512, 2), (200, 3), (4096, 1), (300, 40), (64, 4)])
def test_local_block_backward(L, B, conv, monkeypatch):
    from proteinbert_pytorch_replication_amd.ops import local_track
    from proteinbert_pytorch_replication_amd.ops.local_track import local_block
    monkeypatch.setattr(local_track, "DGRAD_FIN", conv != 5)
    m, blk = make_block(L, seed=1)
    x0 = torch.randn(B, L, 128, device="cuda").to(torch.bfloat16)
    gb0 = torch.randn(B, 128, device="cuda") * 0.5
    dh = torch.randn(B, L, 128, device="cuda")
    dv = torch.randn(B, 512, device="cuda") * 1e-2
    params = [blk.local_narrow_conv_layer[0].weight, blk.local_narrow_conv_layer[0].bias,
              blk.local_wide_conv_layer[0].weight, blk.local_wide_conv_layer[0].bias,
              blk.local_norm_1.weight, blk.local_norm_1.bias, blk.local_linear_layer[0].weight,
              blk.local_linear_layer[0].bias, blk.local_norm_2.weight, blk.local_norm_2.bias]

    x = x0.clone().requires_grad_(True)
    gb = gb0.clone().requires_grad_(True)
    h2, vpart = local_block(x, gb, blk)
    loss = (h2.float() * dh).sum() + (vpart.sum(1) * dv).sum()
    got = torch.autograd.grad(loss, [x, gb] + params)

    xr = x0.float().clone().requires_grad_(True)
    gbr = gb0.clone().requires_grad_(True)
    rh2, rv = torch_local(xr, gbr, blk)
    lr = (rh2 * dh).sum() + (rv * dv).sum()
    ref = torch.autograd.grad(lr, [xr, gbr] + params)
    torch.cuda.synchronize()
    names = ["x", "gb", "wn", "bn", "ww", "bw", "g1", "be1", "wl", "bl", "g2", "be2"]
    errs = {n: rel(a, b) for n, a, b in zip(names, got, ref)}
    print(f"L={L} B={B}: " + " ".join(f"{n}={e:.2e}" for n, e in errs.items()))
    for n, e in errs.items():
        assert e < 3e-2, f"{n}: rel err {e:.3e}"


@pytest.mark.parametrize("B,L,P", [(2, 256, 2), (3, 300, 3)])
def test_cp_halo_conv_kernels_match_whole_sequence(B, L, P):
    """The context-parallel conv launchers (pbx_conv_fwd3x / pbx_conv_dgrad4x / pbx_wgrad2x: neighbour
    rows in place, csrc/conv4.hip, csrc/wgrad.hip) on P shards with 20-row halos reproduce the whole-
    sequence kernels (parallel/cp_fused.py's exchange, done here by slicing)."""
    from proteinbert_pytorch_replication_amd.ops import local_track as lt
    torch.manual_seed(L + P)
    dev = torch.device("cuda")
    H, dil, C = 20, 5, 128
    Ls = L // P
    x = torch.randn(B, L, C, device=dev).to(torch.bfloat16)
    wn, ww = (torch.randn(C, C, 9, device=dev) * 0.05 for _ in range(2))
    bn, bw = torch.randn(C, device=dev) * 0.1, torch.randn(C, device=dev) * 0.1
    gb = torch.randn(B, C, device=dev)
    wpn, wtn = lt.pack_conv(wn)
    wpw, wtw = lt.pack_conv(ww)
    st = lt._lib.stream_ptr(dev)
    T1 = (L + lt.BM1 - 1) // lt.BM1

    def ext(t, r):       # shard r of [B, L, C] with H neighbour rows each side (zeros past the ends)
        z = torch.zeros(B, H, C, dtype=t.dtype, device=dev)
        tp = torch.cat([z, t, z], dim=1)
        return tp[:, r * Ls:r * Ls + Ls + 2 * H].contiguous()

    pre_n, pre_w, s1 = (torch.empty_like(x) for _ in range(3))
    stats = torch.empty(B, T1, 2, device=dev)
    lt.conv_fwd(x, wpn, wpw, bn, bw, gb, pre_n, pre_w, s1, stats, B, L, 9, dil, st)
    ds1 = torch.randn(B, L, C, device=dev).to(torch.bfloat16)
    dx, dpn, dpw = (torch.empty_like(x) for _ in range(3))
    lt.conv_dgrad(ds1, pre_n, pre_w, wtn, wtw, dx, dpn, dpw, B, L, 9, dil, st)
    outs = [(torch.zeros(C, C, 9, device=dev), torch.zeros(C, device=dev)) for _ in range(2)]
    lt._wgrad(dpn, dpw, x, 9, dil, 2, B, L, outs)
    outs_s = [(torch.zeros(C, C, 9, device=dev), torch.zeros(C, device=dev)) for _ in range(2)]
    keep = []
    for r in range(P):
        sl = slice(r * Ls, (r + 1) * Ls)
        xe = ext(x, r)
        pn_s, pw_s, s1_s = (torch.empty(B, Ls, C, dtype=torch.bfloat16, device=dev) for _ in range(3))
        st_s = torch.empty(B, (Ls + lt.BM1 - 1) // lt.BM1, 2, device=dev)
        lt.conv_fwd(xe, wpn, wpw, bn, bw, gb, pn_s, pw_s, s1_s, st_s, B, Ls, 9, dil, st, H, H)
        dx_s, dpn_s, dpw_s = (torch.empty(B, Ls, C, dtype=torch.bfloat16, device=dev) for _ in range(3))
        lt.conv_dgrad(ext(ds1, r), ext(pre_n, r), ext(pre_w, r), wtn, wtw, dx_s, dpn_s, dpw_s, B, Ls, 9, dil, st,
                      H, H)
        keep += lt._wgrad(dpn_s, dpw_s, xe, 9, dil, 2, B, Ls, outs_s, False, H, H)
        torch.cuda.synchronize()
        for name, a, b_ in (("pre_n", pn_s, pre_n[:, sl]), ("pre_w", pw_s, pre_w[:, sl]), ("s1", s1_s, s1[:, sl]),
                            ("dx", dx_s, dx[:, sl]), ("dpn", dpn_s, dpn[:, sl]), ("dpw", dpw_s, dpw[:, sl])):
            assert rel(a, b_) < 1e-2, (name, r, rel(a, b_))
    torch.cuda.synchronize()
    for (dw, db), (dws, dbs) in zip(outs, outs_s):
        assert rel(dws, dw) < 1e-4 and rel(dbs, db) < 1e-4, (rel(dws, dw), rel(dbs, db))


def test_embedding_kernels():
    from proteinbert_pytorch_replication_amd.ops.local_track import EmbedFn
    torch.manual_seed(0)
    E = torch.randn(26, 128, device="cuda", requires_grad=True)
    tok = torch.randint(0, 26, (5, 77), device="cuda")
    out = EmbedFn.apply(tok, E)
    ref = E.detach()[tok]
    assert rel(out, ref) < 4e-3
    g = torch.randn(5, 77, 128, device="cuda")
    (out.float() * g).sum().backward()
    dref = torch.zeros(26, 128, device="cuda").index_add_(0, tok.reshape(-1), g.to(torch.bfloat16).float().reshape(-1, 128))
    assert rel(E.grad, dref) < 1e-5


@pytest.mark.parametrize("B,L,dil", [(3, 300, 5), (2, 512, 5), (1, 130, 2)])
def test_wgrad_token_onehot_vs_fp32(B, L, dil):
    """First-block conv weight gradient through the token one-hot (csrc/wgrad.hip wgrad_tok) vs the fp32
    weight gradient of the 128-channel conv input bf16(E[tok]) (torch.nn.grad.conv1d_weight)."""
    from proteinbert_pytorch_replication_amd.ops.local_track import _wgrad_tok
    torch.manual_seed(B * L)
    V = 26
    E = torch.randn(V, 128, device="cuda")
    tok = torch.randint(0, V, (B, L), device="cuda")
    dpn = torch.randn(B, L, 128, device="cuda").to(torch.bfloat16)
    dpw = torch.randn(B, L, 128, device="cuda").to(torch.bfloat16)
    outs = [(torch.zeros(128, 128, 9, device="cuda"), torch.zeros(128, device="cuda")) for _ in range(2)]
    Wn, Ww = torch.randn(128, 128, 9, device="cuda") * 0.05, torch.randn(128, 128, 9, device="cuda") * 0.05
    dE = torch.zeros(V, 128, device="cuda")
    _wgrad_tok(dpn, dpw, tok, E, dil, B, L, outs, demb=(Wn, Ww, dE))
    torch.cuda.synchronize()
    x = E.to(torch.bfloat16).float()[tok].transpose(1, 2)                       # [B, 128, L]
    dx = torch.zeros(B, 128, L, device="cuda")
    for (dw, db), dp, d, Wc in ((outs[0], dpn, 1, Wn), (outs[1], dpw, dil, Ww)):
        ref = torch.nn.grad.conv1d_weight(x, (128, 128, 9), dp.float().transpose(1, 2), padding=4 * d, dilation=d)
        assert rel(dw, ref) < 1e-5, rel(dw, ref)
        assert rel(db, dp.float().sum(dim=(0, 1))) < 1e-5
        dx += torch.nn.grad.conv1d_input(x.shape, Wc.to(torch.bfloat16).float(), dp.float().transpose(1, 2),
                                         padding=4 * d, dilation=d)
    # the embedding gradient's conv part (first-block fold): sum over positions with token v of conv^T dpre
    dE_ref = torch.zeros(V, 128, device="cuda").index_add_(0, tok.reshape(-1), dx.transpose(1, 2).reshape(-1, 128))
    assert rel(dE, dE_ref) < 1e-5, rel(dE, dE_ref)


@pytest.mark.parametrize("nblocks", [2, 3])
def test_full_model_loss_and_grads_vs_torch(nblocks):
    from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
    from proteinbert_pytorch_replication_amd.ops.fused_model import fused_pretrain_loss
    from proteinbert_pytorch_replication_amd.train.losses import pretrain_loss_torch
    torch.manual_seed(0)
    L, A = 256, 8943
    m = ProteinBERT(sequences_length=L, num_annotations=A, local_dim=128, global_dim=512, key_dim=64, num_heads=4,
                    num_blocks=nblocks, device="cuda", backend="hip")
    X, Y, W = SyntheticUniRefGO(L, A, 6, "cuda", seed=3).next_batch()
    loss = fused_pretrain_loss(m, X, Y, W)
    loss.backward()
    got = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    m.zero_grad(set_to_none=True)
    h, g = m.encode_torch(X["local"], X["global"], torch.float32)
    pl, pg = m.heads_torch(h, g)
    lref = pretrain_loss_torch(pl, pg, Y, {k: v.float() for k, v in W.items()})
    lref.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - lref.item()) < 2e-3 * abs(lref.item())
    norms = {n: p.grad.norm().item() for n, p in m.named_parameters() if p.grad is not None}
    scale = sorted(norms.values())[len(norms) // 2]
    for n, p in m.named_parameters():
        if p.grad is None:
            continue
        err = (got[n].float() - p.grad.float()).norm().item()
        print(f"{n:60s} |g|={norms[n]:.3e} err={err:.3e}")
        # the local-output bias is a softmax-over-batch invariant: its exact gradient
        # is 0, so it is checked against the gradient scale of the model, not relative to itself.
        # Observed on MI355X (profiles/r3u_grad_errors.log): worst relative error 1.8e-2 (bf16 activations)
        assert err < 3e-2 * norms[n] + 1e-4 * scale, f"{n}: err {err:.3e} vs |g| {norms[n]:.3e}"


def test_arena_direct_grads_match_autograd_path():
    """Training path: fused backward accumulates straight into the flat-arena .grad views."""
    from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
    from proteinbert_pytorch_replication_amd.train.optim import FusedAdam
    from proteinbert_pytorch_replication_amd.train.step import PretrainStep
    torch.manual_seed(0)
    L, A = 128, 512
    m = ProteinBERT(sequences_length=L, num_annotations=A, local_dim=128, global_dim=256, key_dim=64, num_heads=4,
                    num_blocks=2, device="cuda", backend="hip")
    opt = FusedAdam(m.parameters(), lr=1e-3)
    step = PretrainStep(m, opt)
    X, Y, W = SyntheticUniRefGO(L, A, 8, "cuda", seed=5).next_batch()
    opt.zero_grad()
    step.loss(X, Y, W).backward()
    direct = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    opt.zero_grad()
    m.backend = "torch"
    step.compute_dtype = torch.float32          # plain fp32 PyTorch oracle (not the bf16 eager path)
    step.loss(X, Y, W).backward()
    ref = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    torch.cuda.synchronize()
    scale = sorted(r.norm().item() for r in ref.values())[len(ref) // 2]
    for n in ref:
        err = (direct[n] - ref[n]).norm().item()
        print(f"{n:60s} |g|={ref[n].norm().item():.3e} err={err:.3e}")
        assert err < 3e-2 * ref[n].norm().item() + 1e-4 * scale, f"{n}: err {err:.3e} |g| {ref[n].norm().item():.3e}"


@pytest.mark.parametrize("arena,det,semantics,L", [(True, False, "reference", 256), (False, False, "reference", 256),
                                                   (True, True, "reference", 256), (True, False, "paper", 256),
                                                   (True, False, "reference", 202)])
def test_embed_fold_matches_data_gradient_path(arena, det, semantics, L, monkeypatch):
    """First block with its conv data gradient folded into the embedding gradient (local_track.EMBED_FOLD:
    pbx_embed_dpre + the E-space conv term of pbx_wgrad_tok) vs conv_dgrad4 + embedding backward: same
    gradients (the fold sums fp32 dS1 + bf16(W)-weighted one-hot sums instead of a bf16-rounded dx)."""
    from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
    from proteinbert_pytorch_replication_amd.ops import local_track
    from proteinbert_pytorch_replication_amd.utils import determinism
    from proteinbert_pytorch_replication_amd.train.optim import FusedAdam
    from proteinbert_pytorch_replication_amd.train.step import PretrainStep
    A = 512                                      # L = 202: 1212 rows, not a multiple of the 256-row tiles
    X, Y, W = SyntheticUniRefGO(L, A, 6, "cuda", seed=9).next_batch()
    grads = []
    monkeypatch.setitem(determinism._STATE, "on", det)       # the fused kernels' fixed-order forms only
    for fold in (False, True):
        monkeypatch.setattr(local_track, "EMBED_FOLD", fold)
        torch.manual_seed(0)
        m = ProteinBERT(sequences_length=L, num_annotations=A, local_dim=128, global_dim=512, key_dim=64,
                        num_heads=4, num_blocks=2, device="cuda", backend="hip", semantics=semantics)
        step = PretrainStep(m, FusedAdam(m.parameters(), lr=1e-3)) if arena else None
        if arena:
            step.optimizer.zero_grad()
            step.loss(X, Y, W).backward()
        else:
            from proteinbert_pytorch_replication_amd.ops.fused_model import fused_pretrain_loss
            fused_pretrain_loss(m, X, Y, W).backward()
        from proteinbert_pytorch_replication_amd.ops import streams
        streams.join()
        torch.cuda.synchronize()
        grads.append({n: p.grad.detach().float().clone() for n, p in m.named_parameters() if p.grad is not None})
    g0, g1 = grads
    assert set(g0) == set(g1)
    for n in g0:
        err = (g0[n] - g1[n]).norm().item()
        ref = g0[n].norm().item()
        print(f"{n:60s} |g|={ref:.3e} err={err:.3e}")
        # outside deterministic mode the block-0 broadcast-gradient column sums use fp32 atomics (order noise
        # ~1e-10, tools/probe_conv_det.py) that can flip a bf16 rounding downstream of them
        tol = 2e-2 if n == "local_embedding.weight" else (1e-3 if det else 1e-2)
        assert err <= tol * ref + 1e-6, (n, err, ref)


@pytest.mark.parametrize("L,B", [(512, 4), (300, 3), (64, 5)])
def test_dgrad_fin_matches_separate_finalize(L, B, monkeypatch):
    """conv_dgrad4 with the LN1 backward finalize fused in (local_track.DGRAD_FIN) vs ln1_finalize +
    conv_dgrad4: the same dS1 formula and bf16 rounding, so the block's gradients agree to float-atomic
    order (dgb column sums)."""
    from proteinbert_pytorch_replication_amd.ops import local_track
    from proteinbert_pytorch_replication_amd.ops.local_track import local_block
    m, blk = make_block(L, seed=3)
    torch.manual_seed(L + B)
    x0 = torch.randn(B, L, 128, device="cuda").to(torch.bfloat16)
    gb0 = torch.randn(B, 128, device="cuda") * 0.5
    dh = torch.randn(B, L, 128, device="cuda")
    dv = torch.randn(B, 512, device="cuda") * 1e-2
    params = [blk.local_narrow_conv_layer[0].weight, blk.local_wide_conv_layer[0].weight, blk.local_norm_1.weight,
              blk.local_norm_1.bias, blk.local_linear_layer[0].weight]
    out = []
    for fin in (False, True):
        monkeypatch.setattr(local_track, "DGRAD_FIN", fin)
        x = x0.clone().requires_grad_(True)
        gb = gb0.clone().requires_grad_(True)
        h2, vpart = local_block(x, gb, blk)
        loss = (h2.float() * dh).sum() + (vpart.sum(1) * dv).sum()
        out.append(torch.autograd.grad(loss, [x, gb] + params))
    torch.cuda.synchronize()
    for n, a, b in zip(["x", "gb", "wn", "ww", "g1", "be1", "wl"], *out):
        assert rel(b, a) < 2e-3, f"{n}: {rel(b, a):.3e}"


@pytest.mark.parametrize("B,L", [(3, 512), (2, 300)])
def test_conv_fwd_token_gather_matches_embedding_input(B, L):
    """The first block's conv with the embedding gathered in its staging pass (pbx_conv_fwd3t) writes the
    same s1 / GELU' / LayerNorm partials, bitwise, as conv_fwd3 over the materialised bf16(E[tok])."""
    from proteinbert_pytorch_replication_amd.ops import _lib
    from proteinbert_pytorch_replication_amd.ops.local_track import BM1, conv_fwd, pack_conv
    torch.manual_seed(B * L)
    dev = "cuda"
    E = torch.randn(26, 128, device=dev)
    tok = torch.randint(0, 26, (B, L), device=dev)
    wn, ww = torch.randn(128, 128, 9, device=dev) * 0.05, torch.randn(128, 128, 9, device=dev) * 0.05
    bn, bw, gb = torch.randn(128, device=dev), torch.randn(128, device=dev), torch.randn(B, 128, device=dev)
    (wpn, _), (wpw, _) = pack_conv(wn), pack_conv(ww)
    T1 = (L + BM1 - 1) // BM1
    outs = []
    for gather in (False, True):
        o = [torch.empty(B, L, 128, dtype=torch.bfloat16, device=dev) for _ in range(3)]
        st1 = torch.empty(B, T1, 2, device=dev)
        st = _lib.stream_ptr(torch.device(dev))
        if gather:
            eb = E.to(torch.bfloat16).contiguous()
            _lib.call("pbx_conv_fwd3t", tok.data_ptr(), eb.data_ptr(), wpn.data_ptr(), wpw.data_ptr(), bn.data_ptr(),
                      bw.data_ptr(), gb.data_ptr(), o[0].data_ptr(), o[1].data_ptr(), o[2].data_ptr(), st1.data_ptr(),
                      B, L, 9, 5, st)
        else:
            x = E.to(torch.bfloat16)[tok].contiguous()
            # conv_fwd3 itself (conv_fwd picks the persistent conv_fwd5 for dilation 5: same s1 / GELU'
            # images, LayerNorm partials summed in another order -- checked below)
            _lib.call("pbx_conv_fwd3x", x.data_ptr(), wpn.data_ptr(), wpw.data_ptr(), bn.data_ptr(), bw.data_ptr(),
                      gb.data_ptr(), o[0].data_ptr(), o[1].data_ptr(), o[2].data_ptr(), st1.data_ptr(), B, L, 9, 5,
                      0, 0, st)
            o5 = [torch.empty_like(t) for t in o]
            st5 = torch.empty_like(st1)
            conv_fwd(x, wpn, wpw, bn, bw, gb, o5[0], o5[1], o5[2], st5, B, L, 9, 5, st)
        outs.append(o + [st1])
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    for a, b in zip(o5, outs[0][:3]):
        assert torch.equal(a, b)
    torch.testing.assert_close(st5, outs[0][3], rtol=2e-5, atol=2e-5 * L * 128)
