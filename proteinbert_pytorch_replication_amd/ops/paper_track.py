"""Paper-semantics block pieces on MI355X: fused local track (``csrc/paper_local.hip`` + the
semantics-independent conv kernels) and the row-softmax local head loss.

``semantics="paper"`` is the published ProteinBERT (per-position LayerNorm over channels with a
``[C]`` affine, attention softmax over positions, local softmax over the vocabulary); reference
``ProteinBERT/modules.py:148-164,212-217`` normalises over ``(L, C)`` instead.
One :class:`PaperBlockFn` is::

    s1 = x + GELU(conv_d1(x)) + GELU(conv_d5(x)) + gb        (conv_fwd3, shared with reference semantics)
    h1 = LN_C(s1); s2 = h1 + GELU(h1 Wl^T + bl); h2 = LN_C(s2)  (pbx_pc_ln_linear_fwd: 1 launch)

    o  = attention(h2, g) over positions                       (K/V GEMM + split-L HIP core)

and its backward is the attention core + two GEMMs, one LayerNorm/MLP launch (recomputing h1 / the
MLP pre-activation from s1, both h2 gradients as inputs) and the conv data / weight gradient
kernels.  The global track runs through the fused global-track kernels.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib, streams
from ..train.arena import notify_grads_ready
from .gemm import gemm as _gemm
from .global_track import (BF16, F32, _Grads, _UNIT_LOSS_GRAD, bf16_of, go_head_backward, go_head_forward,
                           loss_total, mm32, addmm_into)
from .local_track import (CH, conv_dgrad, conv_fwd, conv_tile, dwl_slab, pack_conv, _grad_dst, _wgrad,
                          _wgrad_tok, embed_fold_bwd, wgrad_tok_ok)

_P, _I, _F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
_lib.register("pbx_pc_ln_linear_fwd", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _F, _P])
_lib.register("pbx_pc_ln_linear_bwd", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                       _P, _P, _I, _I, _I, _P])
_lib.register("pbx_pa_fused_fwd", [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P])
_lib.register("pbx_paper_head", [_P, _P, _P, _P, _P, _P, _P, _P, _P, ctypes.c_long, _I, _F, _P])
_lib.register("pbx_paper_head_parts", [ctypes.c_long])
_lib.register("pbx_pa_fused_bwd", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P])
# fp32 query-path GEMMs with fused layouts / epilogues (csrc/sgemm.hip)
_lib.register("pbx_sg_query_fwd", [_P, _P, _P, _P, _P, _I, _I, _I, _I, _F, _P])
_lib.register("pbx_sg_query_dg", [_P, _P, _P, _P, _P, _I, _I, _I, _I, _F, _P])
_lib.register("pbx_sg_query_dwq", [_P, _P, _P, _P, _P, _I, _I, _I, _I, _F, _P])
_lib.register("pbx_sg_query_ws", [_I, _I, _I, _I])
_lib.register("pbx_pa_wimg", [_P, _P, _P, _I, _I, _I, _I, _P])
_lib.register("pbx_group_colsum", [_P, _I, _I, _I, _P, _P])


def group_colsum(t: torch.Tensor) -> torch.Tensor:
    """``[G, R, C]`` fp32 -> ``[G, C]``, summed over R in order (``csrc/glob.hip``)."""
    G, R, C = t.shape
    if t.device.type != "cuda":
        return t.sum(dim=1)
    t = t.contiguous()
    out = torch.empty((G, C), dtype=F32, device=t.device)
    _lib.call("pbx_group_colsum", t.data_ptr(), G, R, C, out.data_ptr(), _lib.stream_ptr(t.device))
    return out
_lib.register("pbx_pa_dwkv_add", [_P, _P, _P, _I, _I, _I, _I, _P])


def _sg_ws(B: int, G: int, H: int, K: int, dev) -> torch.Tensor:
    """Split-K partial-sum workspace of the query-path GEMMs (csrc/sgemm.hip)."""
    return torch.empty(_lib.lib().pbx_sg_query_ws(B, G, H, K), dtype=torch.float32, device=dev)

# paper attention form: "fused" (csrc/paper_fused.hip: K/V projections on MFMA inside the attention
# kernels, no [B*L, H*(K+VD)] pre-activation tensor; H in {2, 4}); other head counts take "split" (in-tree
# K/V GEMM + csrc/paper_attn.hip core; tests force it to check the fallback)
PAPER_ATTN = "fused"
FUSED_CHUNK_F = 256                         # positions per forward work item
FUSED_BWD_WAVES = 8                         # backward: 32 positions per wave

LN_EPS = 1e-5
TR = 32          # positions per work item of the paper LayerNorm kernels


class PaperBlockFn(torch.autograd.Function):
    """Fused local track + local->global attention of one block, paper semantics.

    Outputs ``h2`` (the block's local output, bf16 ``[B, L, 128]``) and ``o`` (the attention output,
    fp32 ``[B, H*VD]``, consumed unscaled by the global track).  The attention is the published one:
    ``q = tanh(g Wq) / sqrt(K)``, ``pre = h2 [Wk | Wv]`` (one library GEMM), then the split-L HIP core
    (``csrc/paper_attn.hip``: tanh keys, GELU values, pad-masked softmax over positions).  In the
    backward both gradients of ``h2`` (from the next block and from the attention projection) enter
    the LayerNorm/MLP kernel as two inputs, so they are never summed in a separate pass.
    """

    @staticmethod
    def forward(ctx, x, gb, g, wn, bn, ww, bw, g1, be1, wl, bl, g2, be2, Wq, Wk, Wv, mask, dil: int, packed=None,
                tok=None, emb=None, emb_grad: bool = False, cp=None):
        from .paper_attention import KEY_DIM, VALUE_DIM, _nsplit
        params = (wn, bn, ww, bw, g1, be1, wl, bl, g2, be2, Wq, Wk, Wv)
        B, L, C = x.shape
        assert C == CH and x.dtype == BF16 and x.is_contiguous()
        assert g1.shape == (CH,), "paper semantics: LayerNorm affine is [C]"
        H, _, K = Wk.shape
        VD = Wv.shape[2]
        assert K == KEY_DIM and VD == VALUE_DIM
        KS = wn.shape[2]
        dev = x.device
        stream = _lib.stream_ptr(dev)
        BM1 = conv_tile(L)
        T1 = (L + BM1 - 1) // BM1
        if packed is not None:
            wpn, wtn, wpw, wtw = packed
        else:
            wpn, wtn = pack_conv(wn)
            wpw, wtw = pack_conv(ww)
        wl_b = bf16_of(wl)
        gb = gb.detach().float().contiguous()
        pre_n, pre_w, s1 = torch.empty_like(x), torch.empty_like(x), torch.empty_like(x)
        st1 = torch.empty((B, T1, 2), dtype=F32, device=dev)       # whole-sequence partials (unused here)
        # cp (parallel/cp_fused.py CPShard): x is this rank's slice; the convs read the neighbours' halo
        # rows (P2P), LayerNorm is per position (nothing else to exchange in the local track)
        x_ext, hlo = (x, 0) if cp is None else (cp.halo_rows(x), cp.halo)
        if cp is not None and (tok is not None or emb_grad):
            raise ValueError("context parallelism: the token-embedding first-block forms are single-shard only")
        conv_fwd(x_ext, wpn, wpw, bn, bw, gb, pre_n, pre_w, s1, st1, B, L, KS, dil, stream, hlo, hlo)
        h2 = torch.empty_like(x)
        stats = torch.empty((B * L, 4), dtype=F32, device=dev)
        _lib.call("pbx_pc_ln_linear_fwd", s1.data_ptr(), g1.data_ptr(), be1.data_ptr(), wl_b.data_ptr(),
                  bl.data_ptr(), g2.data_ptr(), be2.data_ptr(), h2.data_ptr(), stats.data_ptr(), B, L, LN_EPS, stream)
        # attention: q from the global track, K/V projection as one library GEMM, split-L core
        gf = g.detach().float().contiguous()
        # q = tanh(g Wq) at fp32 (the query feeds the softmax over L, so bf16 rounding is kept out of it):
        # one fp32 GEMM reading Wq [H, G, K] in place, tanh and the 1/sqrt(K) scale in its epilogue
        wq32 = Wq.detach().float().contiguous()                                         # [H, G, K]
        G = gf.shape[1]
        q = torch.empty((B, H, K), dtype=F32, device=dev)
        qs = torch.empty((B, H, K), dtype=F32, device=dev)
        _lib.call("pbx_sg_query_fwd", gf.data_ptr(), wq32.data_ptr(), q.data_ptr(), qs.data_ptr(),
                  _sg_ws(B, G, H, K, dev).data_ptr(), B, G, H, K, 1.0 / math.sqrt(K), stream)
        o = torch.empty(B, H * VD, device=dev, dtype=F32)
        lse = torch.empty(B * H, device=dev, dtype=F32)
        mk = None if mask is None else mask.contiguous()
        fused = PAPER_ATTN == "fused" and H in (2, 4)
        if fused:
            # [H][Wk_h^T (64 rows) | Wv_h^T (128 rows)][C] bf16: the MFMA A/B rows of the fused kernels
            wimg = torch.empty((H, K + VD, C), dtype=BF16, device=dev)
            _lib.call("pbx_pa_wimg", Wk.detach().float().contiguous().data_ptr(),
                      Wv.detach().float().contiguous().data_ptr(), wimg.data_ptr(), H, C, K, VD, stream)
            ns = -(-L // FUSED_CHUNK_F)
            part = torch.empty(B * H, ns, 2 + VD, device=dev, dtype=F32)
            _lib.call("pbx_pa_fused_fwd", h2.data_ptr(), wimg.data_ptr(), qs.data_ptr(), _lib.ptr(mk),
                      part.data_ptr(), o.data_ptr(), lse.data_ptr(), B, L, H, stream)
            wsave, pre = wimg, None
        else:
            wcat = torch.cat([Wk.detach().permute(1, 0, 2).reshape(C, H * K),
                              Wv.detach().permute(1, 0, 2).reshape(C, H * VD)], dim=1).to(BF16)   # [C, H*(K+VD)]
            pre = mm32(h2.view(B * L, C), wcat).to(BF16)                                  # [R, N] bf16
            ns = _nsplit(B, H, L)
            part = torch.empty(B * H, ns, 2 + VD, device=dev, dtype=F32)
            _lib.call("pbx_paper_attn_fwd", pre.data_ptr(), qs.data_ptr(), _lib.ptr(mk), part.data_ptr(),
                      o.data_ptr(), lse.data_ptr(), B, L, H, K, VD, ns, stream)
            wsave = wcat
        if cp is not None:
            o, lse = _cp_softmax_combine(o, lse, B, H, VD, cp)
        ctx.fused = fused
        # the first block: x = bf16(emb[tok]), the conv weight gradient goes through the token one-hot
        ctx.tok = (tok, emb) if wgrad_tok_ok(tok, emb, L, KS) else None
        # emb_grad: x has no autograd history; the backward folds the conv data gradient into emb's
        # gradient (local_track.EMBED_FOLD)
        ctx.emb_grad = bool(emb_grad)
        if ctx.emb_grad and (ctx.tok is None or x.requires_grad):
            raise ValueError("emb_grad needs a token-embedding input without autograd history (wgrad_tok_ok)")
        # gf (the fp32 g of the dWq product) is saved through autograd: when g is already fp32 it is an alias
        # of g, and the version check then catches an in-place change of g before backward
        ctx.save_for_backward(x_ext, pre_n, pre_w, s1, stats, wtn, wtw, wl_b, q, qs, wsave, pre, mk, o, lse,
                              h2, wq32, gf)
        ctx.cp, ctx.hlo = cp, hlo
        ctx.meta = (B, L, KS, dil, BM1, H, K, VD, ns)
        ctx.params = params
        ctx.set_materialize_grads(False)
        return h2, o

    @staticmethod
    def backward(ctx, dh2, do):
        (x_ext, pre_n, pre_w, s1, stats, wtn, wtw, wl_b, q, qs, wsave, pre, mk, o, lse, h2,
         wq32, gf32) = ctx.saved_tensors
        B, L, KS, dil, BM1, H, K, VD, ns = ctx.meta
        cp, hlo = ctx.cp, ctx.hlo
        x = x_ext if cp is None else x_ext[:, hlo:hlo + L]     # this shard's rows (shape / dtype only)
        dev = x.device
        stream = _lib.stream_ptr(dev)
        params = ctx.params
        wn, bn, ww, bw, g1, be1, wl, bl, g2, be2, Wq, Wk, Wv = params
        dsts = [_grad_dst(p, p.shape) for p in params]
        (dwn, _), (dbn, _), (dww, _), (dbw, _), (dg1, _), (dbe1, _), (dwl, _), (dbl, _), (dg2, _), (dbe2, _) = dsts[:10]
        (dWq, _), (dWk, _), (dWv, _) = dsts[10:]
        R, C = B * L, CH
        dh2 = None if dh2 is None else dh2.to(BF16).contiguous()
        dg = None
        dh2_att = [None, None]
        if do is not None:
            dO = do.float().contiguous()
            if ctx.fused:
                # keys / values recomputed on MFMA; dh2 per head pair, dpre rows for the dW GEMM
                npair = H // 2
                dh2p = torch.empty((npair, B, L, C), dtype=BF16, device=dev)
                dpre = torch.empty((R, H * (K + VD)), dtype=BF16, device=dev)
                nsb = -(-L // (32 * FUSED_BWD_WAVES))
                dq_part = torch.empty(B * H, nsb, K, device=dev, dtype=F32)
                _lib.call("pbx_pa_fused_bwd", h2.data_ptr(), wsave.data_ptr(), qs.data_ptr(), _lib.ptr(mk),
                          lse.data_ptr(), o.data_ptr(), dO.data_ptr(), dh2p.data_ptr(), dpre.data_ptr(),
                          dq_part.data_ptr(), B, L, H, FUSED_BWD_WAVES, stream)
                dh2_att = [dh2p[i] for i in range(npair)] + [None] * (2 - npair)
            else:
                dpre = torch.empty_like(pre)
                dq_part = torch.empty(B * H, ns, K, device=dev, dtype=F32)
                _lib.call("pbx_paper_attn_bwd", pre.data_ptr(), qs.data_ptr(), _lib.ptr(mk), lse.data_ptr(),
                          o.data_ptr(), dO.data_ptr(), dpre.data_ptr(), dq_part.data_ptr(), B, L, H, K, VD, ns,
                          stream)
                dh2_att = [mm32(dpre, wsave.t()).to(BF16), None]                          # [R, C] bf16
            dqs = group_colsum(dq_part).view(B, H, K)
            if cp is not None:
                cp.all_reduce_(dqs)             # q is replicated: its gradient sums every shard's positions
            G = gf32.shape[1]
            # dg = dqpre Wq^T with dqpre = dqs (1 - q^2) / sqrt(K) formed while the operand is staged
            dg = torch.empty((B, G), dtype=F32, device=dev)
            _lib.call("pbx_sg_query_dg", dqs.data_ptr(), q.data_ptr(), wq32.data_ptr(), dg.data_ptr(),
                      _sg_ws(B, G, H, K, dev).data_ptr(), B, G, H, K, 1.0 / math.sqrt(K), stream)

            def att_wgrad(dpre=dpre, h2=h2, dqs=dqs, q=q, gf32=gf32):
                # attention projection weight gradients: dWk | dWv = h2^T dpre (K = B*L), dWq = g^T dqpre
                # in-tree MFMA GEMM, deterministic split-K over the K = B*L rows (csrc/gemm.hip)
                dwcat = torch.empty((C, dpre.shape[1]), dtype=F32, device=dev)
                _gemm(h2.reshape(R, C), dpre, dwcat, ta=True, tb=False)                   # [C, N] fp32
                if dWk.is_contiguous() and dWv.is_contiguous():
                    _lib.call("pbx_pa_dwkv_add", dwcat.data_ptr(), dWk.data_ptr(), dWv.data_ptr(), H, C, K, VD,
                              _lib.stream_ptr(dev))
                else:
                    dWk.add_(dwcat[:, :H * K].view(C, H, K).permute(1, 0, 2))
                    dWv.add_(dwcat[:, H * K:].view(C, H, VD).permute(1, 0, 2))
                # dWq += g^T dqpre, accumulated into the [H, G, K] gradient (fp32, fixed-order split-K)
                ws = _sg_ws(B, G, H, K, dev)
                _lib.call("pbx_sg_query_dwq", gf32.data_ptr(), dqs.data_ptr(), q.data_ptr(), dWq.data_ptr(),
                          ws.data_ptr(), B, G, H, K, 1.0 / math.sqrt(K), _lib.stream_ptr(dev))
                return [dwcat, ws]

            if streams.ENABLED and dev.type == "cuda" and all(d for _, d in dsts[10:]):
                # only the optimizer and the DP all-reduce read them: beside the critical path, on the
                # weight-gradient stream (the split-K GEMM over B*L rows was ~60 us per block on it)
                streams.launch(dev, att_wgrad, keep=[dpre, h2, dqs, q, gf32], name="wgrad")
            else:
                att_wgrad()
        ds1 = torch.empty_like(x)
        T = (L + TR - 1) // TR
        dgbp = torch.empty((B, T, CH), dtype=F32, device=dev)
        _lib.call("pbx_pc_ln_linear_bwd", _lib.ptr(dh2), _lib.ptr(dh2_att[0]), _lib.ptr(dh2_att[1]),
                  s1.data_ptr(), stats.data_ptr(),
                  g1.data_ptr(), be1.data_ptr(), wl_b.data_ptr(), bl.data_ptr(), g2.data_ptr(), ds1.data_ptr(),
                  dgbp.data_ptr(), dg2.data_ptr(), dbe2.data_ptr(), dg1.data_ptr(), dbe1.data_ptr(), dwl.data_ptr(),
                  dbl.data_ptr(), *dwl_slab(dev), B, L, stream)
        dgb = group_colsum(dgbp)
        if cp is not None:
            cp.all_reduce_(dgb)                 # gb is replicated: its gradient sums every shard's positions
        dpn, dpw = torch.empty_like(x), torch.empty_like(x)
        demb, dE_direct, dx = None, True, None
        if ctx.emb_grad:
            demb, dE_direct = embed_fold_bwd(*ctx.tok, ds1, pre_n, pre_w, dpn, dpw, wn, ww, stream)
        elif cp is None:
            dx = torch.empty_like(x)
            conv_dgrad(ds1, pre_n, pre_w, wtn, wtw, dx, dpn, dpw, B, L, KS, dil, stream)
        else:
            dx = torch.empty_like(x)
            conv_dgrad(*cp.halo_rows_many(ds1, pre_n, pre_w), wtn, wtw, dx, dpn, dpw, B, L, KS, dil, stream,
                       hlo, hlo)
        if ctx.tok is not None:
            tok, emb = ctx.tok
            wg = lambda: _wgrad_tok(dpn, dpw, tok, emb, dil, B, L, [(dwn, dbn), (dww, dbw)], demb)   # noqa: E731
        else:
            wg = lambda: _wgrad(dpn, dpw, x_ext, KS, dil, 2, B, L, [(dwn, dbn), (dww, dbw)],   # noqa: E731
                                xlo=hlo, xhi=hlo)
        if all(dsts[i][1] for i in (0, 1, 2, 3)) and dE_direct and streams.ENABLED:
            streams.launch(dev, wg, keep=[dpn, dpw, x_ext] + ([demb[2]] if demb is not None else []), name="wgrad")
        else:
            wg()
        direct = [p for p, (_, d) in zip(params, dsts) if d]
        if demb is not None and dE_direct:
            direct.append(ctx.tok[1])
        if direct:
            notify_grads_ready(direct)
        pgrads = [None if d else gr for (gr, d) in dsts]
        gemb = demb[2] if demb is not None and not dE_direct else None
        return (dx, dgb, dg, *pgrads, None, None, None, None, gemb, None, None)


def _cp_softmax_combine(o: torch.Tensor, lse: torch.Tensor, B: int, H: int, VD: int, cp):
    """Merge the shards' softmax-over-positions results: each rank's ``(o_r, lse_r)`` covers its own
    positions; the group's is ``lse = logsumexp_r lse_r`` and ``o = sum_r exp(lse_r - lse) o_r`` (one MAX
    and one SUM all-reduce of ``B H (1 + VD)`` floats).  With the group's ``(o, lse)`` the backward kernel
    is exact on each shard's positions.  A shard whose positions of a sample are all padding carries
    ``lse = +inf`` (the kernels' "no mass" value: p = exp(s - lse) = 0) and adds nothing."""
    import torch.distributed as dist
    empty = torch.isposinf(lse)
    lr = torch.where(empty, torch.full_like(lse, -float("inf")), lse)
    m = lr.clone()
    dist.all_reduce(m, op=dist.ReduceOp.MAX, group=cp.group)
    mz = torch.where(torch.isfinite(m), m, torch.zeros_like(m))
    w = torch.exp(lr - mz)                                                  # 0 for an all-padding shard
    ow = torch.where(w[:, None] > 0, o.view(B * H, VD) * w[:, None], torch.zeros_like(o.view(B * H, VD)))
    s = torch.cat([w, ow.reshape(-1)])
    dist.all_reduce(s, group=cp.group)
    sw = s[:B * H]
    has = sw > 0
    o_g = torch.where(has[:, None], s[B * H:].view(B * H, VD) / sw.clamp_min(1e-30)[:, None], 0.0)
    lse_g = torch.where(has, mz + torch.log(sw.clamp_min(1e-30)), torch.full_like(sw, float("inf")))
    return o_g.reshape(B, H * VD).contiguous(), lse_g.contiguous()


def paper_block(x: torch.Tensor, gb: torch.Tensor, g: torch.Tensor, blk, mask, packed=None, tok=None, emb=None,
                emb_grad: bool = False, cp=None):
    """``(h2, o)`` of one paper-semantics block's local track + attention (fused HIP path); ``tok`` /
    ``emb``: ``x`` is the token embedding bf16(emb[tok]) (the first block); ``emb_grad``: the backward
    returns ``emb``'s gradient (``x`` without autograd history, local_track.EMBED_FOLD)."""
    nc = blk.local_narrow_conv_layer[0]
    wc = blk.local_wide_conv_layer[0]
    att = blk.global_attention_layer
    return PaperBlockFn.apply(x, gb, g, nc.weight, nc.bias, wc.weight, wc.bias, blk.local_norm_1.weight,
                              blk.local_norm_1.bias, blk.local_linear_layer[0].weight,
                              blk.local_linear_layer[0].bias, blk.local_norm_2.weight, blk.local_norm_2.bias,
                              att.Wq, att.Wk, att.Wv, mask, blk.wide_conv_dilation, packed, tok, emb, emb_grad, cp)


def paper_local_block(x: torch.Tensor, gb: torch.Tensor, blk, packed=None) -> torch.Tensor:
    """Local track only (``h2``); the attention output is dropped (tests / encoders without the
    global track's consumer)."""
    g = torch.zeros((x.shape[0], blk.global_dim), dtype=F32, device=x.device)
    h2, _ = paper_block(x, gb, g, blk, None, packed)
    return h2


_ONES = {}


def unit_attention_weight(K: int, device) -> torch.Tensor:
    """Constant ``[K]`` ones: the fused global-track kernels scale the attention input by
    ``sum(W_parameter) / K`` (reference semantics); in paper semantics the attention output enters
    the global track unscaled and ``W_parameter`` is unused (as in ``GlobalAttention.forward_paper``)."""
    key = (K, str(device))
    t = _ONES.get(key)
    if t is None:
        t = torch.ones(K, dtype=F32, device=device)
        _ONES[key] = t
    return t


class PaperHeadsLossFn(torch.autograd.Function):
    """Both heads + the paper-semantics loss: local head softmax over the vocabulary (NLL of the
    target residue, weighted, mean over B*L), GO head sigmoid + BCE (the reference's, ``utils.py:294``).
    Gradients are produced in the forward pass (the loss is terminal)."""

    @staticmethod
    def forward(ctx, h, g2, g2_bf, wo, bo, wa, ba, y_l, y_g, w_l, w_g):
        dev = h.device
        st = _lib.stream_ptr(dev)
        B, L, C = h.shape
        V = wo.shape[0]
        A = wa.shape[0]
        loss = torch.empty(2, dtype=F32, device=dev)        # each head writes its slot (pbx_colsum_set)
        R = B * L
        hb = h.reshape(R, C)
        # one launch (csrc/phead.hip): logits, row softmax over V, weighted NLL, dZ, dh = dZ Wo, bias-gradient
        # and loss partials; dWo = dZ^T h is the in-tree split-K GEMM over the K = B*L rows
        parts = _lib.lib().pbx_paper_head_parts(R)
        dh = torch.empty((B, L, C), dtype=BF16, device=dev)
        dzl = torch.empty((R, 32), dtype=BF16, device=dev)
        dbo_part = torch.empty((parts, V), dtype=F32, device=dev)
        loss_part = torch.empty(parts, dtype=F32, device=dev)
        y = y_l.reshape(-1).contiguous()
        wl = w_l.reshape(-1).float().contiguous()
        _lib.call("pbx_paper_head", hb.data_ptr(), wo.detach().float().contiguous().data_ptr(),
                  bo.detach().float().contiguous().data_ptr(), y.data_ptr(), wl.data_ptr(), dh.data_ptr(),
                  dzl.data_ptr(), dbo_part.data_ptr(), loss_part.data_ptr(), R, V, 1.0 / float(R), st)
        _lib.call("pbx_colsum_set", loss_part.data_ptr(), parts, 1, loss.data_ptr(), None, st)
        dbo = torch.empty(V, dtype=F32, device=dev)
        _lib.call("pbx_colsum_set", dbo_part.data_ptr(), parts, V, dbo.data_ptr(), None, st)
        dwo32 = torch.empty((32, C), dtype=F32, device=dev)
        _gemm(dzl, hb, dwo32, ta=True, tb=False)                                            # K = B*L: split-K
        dwo = dwo32[:V]
        dz, dba, gx = go_head_forward(g2_bf, wa, ba, y_g, w_g, loss[1:])
        ctx.save_for_backward(dh, dwo, dbo, dz, dba, gx)
        ctx.params = (wo, bo, wa, ba)
        ctx.mark_non_differentiable(loss)
        ctx.set_materialize_grads(False)
        return loss_total(loss), loss

    @staticmethod
    def backward(ctx, dtotal, _dparts):
        dh, dwo, dbo, dz, dba, g2_bf = ctx.saved_tensors
        wo, bo, wa, ba = ctx.params
        if dtotal is None:
            return (None,) * 11
        gr = _Grads([wo, bo, wa, ba])
        dwo_d, dbo_d, dwa_d, dba_d = gr.dst
        if _UNIT_LOSS_GRAD[0]:
            s = None
            dh_s = dh
        else:
            s = dtotal.reshape(1).to(F32).contiguous()
            dh_s = (dh.float() * s.reshape(())).to(dh.dtype)
        # dst += s * src as one-row folds (in-tree, csrc/glob.hip)
        st = _lib.stream_ptr(dh.device)
        _lib.call("pbx_colsum_add", dwo.data_ptr(), 1, dwo.numel(), dwo_d.data_ptr(), _lib.ptr(s), st)
        _lib.call("pbx_colsum_add", dbo.data_ptr(), 1, dbo.numel(), dbo_d.data_ptr(), _lib.ptr(s), st)
        dg2 = go_head_backward(dz, dba, g2_bf, wa, dwa_d, dba_d, s)
        return (dh_s, dg2, None, *gr.finish(), None, None, None, None)
