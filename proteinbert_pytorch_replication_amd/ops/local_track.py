"""Autograd wrappers of the fused CDNA4 local-track kernels (``csrc/conv2.hip``, ``csrc/conv4.hip``,
``csrc/wgrad.hip``, ``csrc/ln.hip``, ``csrc/pool.hip``).

One :class:`LocalBlockFn` call is the whole local track of one ``ProteinBERTBlock`` in reference
semantics (reference ``ProteinBERT/modules.py:201-219``)::

    s1 = x + GELU(conv_d1(x)) + GELU(conv_d5(x)) + gb       (conv_fwd3: 1 launch)
    h1 = LN_(L,C)(s1); s2 = h1 + GELU(h1 Wl^T + bl)           (ln_linear_fwd: 1 launch)
    h2 = LN_(L,C)(s2); vpart = sum_tile GELU(h2 Wv_cat^T)     (pool_fwd, csrc/pool.hip: 1 launch)

and its backward is 6-7 launches on the main stream (attention pool with GELU' recomputed + LN2
partials, LN2 constants, LN2 + MLP, conv data gradient with the LN1 finalize fused in) plus the conv
weight gradient, its slab fold and the MLP dW fold on the weight-gradient stream.  Activations are bf16
``[B, L, 128]`` channels-last; parameters stay fp32 masters and are packed to bf16 kernel layouts
once per forward.  The global track (``[B, 512]`` vectors) is :mod:`.global_track`.

Every op raises if the HIP library is missing — there is no silent eager fallback on a GPU.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Dict, Optional, Tuple

import torch

from . import _lib, streams
from ..train.arena import notify_grads_ready
from ..utils.determinism import fused_deterministic
from .global_track import bf16_of

_P, _I, _F, _L = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_long

_lib.register("pbx_conv_fwd3x", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P])
_lib.register("pbx_conv_fwd5x", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P])
_lib.register("pbx_conv_dgrad4x", [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P])
_lib.register("pbx_wgrad2x", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P])
_lib.register("pbx_pack_conv_frag", [_P, _P, _P, _I, _P])
_lib.register("pbx_wgrad2", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P])
_lib.register("pbx_wgrad_tok", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P])
_lib.register("pbx_ln_linear_fwd", [_P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _I, _I, _F, _P])
_lib.register("pbx_pool_fwd", [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _F, _P])
_lib.register("pbx_pool_bwd", [_P, _P, _P, _P, _P, _I, _P, _P, _P, _I, _I, _I, _P])
_lib.register("pbx_ln2_linear_bwd", [_P, _P, _P, _P, _I, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P,
                                     _P, _P, _P, _P, _P, _I, _I, _F, _P, _I, _I, _I, _I, _P])
_lib.register("pbx_ln2_bwd_slab_rows", [_I, _I, _I])
_lib.register("pbx_colsum_add", [_P, _I, _I, _P, _P, _P])
_lib.register("pbx_colsum_add2", [_P, _I, _P, _P, _I, _P, _I, _P])
_lib.register("pbx_ln1_finalize", [_P, _P, _P, _I, _I, _P, _I, _P, _P, _P, _I, _I, _F, _I, _P])
_lib.register("pbx_embed_fwd", [_P, _P, _P, _L, _P])
_lib.register("pbx_embed_bwd", [_P, _P, _P, _L, _I, _P, _P])
_lib.register("pbx_conv_fwd3t", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P])
_lib.register("pbx_conv_dgrad4f", [_P, _P, _P, _I, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I,
                                    _F, _P])
_lib.register("pbx_embed_dpre", [_P, _P, _P, _P, _P, _P, _P, _L, _I, _P, _P])
_lib.register("pbx_embed_bwd_groups", [_L])

CH = 128          # kernels are specialised for local_dim = 128
PB = 32           # positions per workgroup of the position-major LayerNorm kernels
LN_EPS = 1e-5     # nn.LayerNorm default (reference modules.py:148-164)


BM1 = 128         # positions per conv-forward workgroup (= the tile of the LayerNorm-1 partials)
def attn_pool_supported(NJ: int) -> bool:
    """The attention-pool kernels are built for H * value_dim = NJ in (256, 512)."""
    return NJ in (256, 512)


def conv_tile(L: int) -> int:
    return BM1


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


# the conv forward: the persistent software-pipelined kernel (csrc/conv5.hip, dilation 5) or conv_fwd3
# (csrc/conv2.hip, any dilation; also the first block's token-gather form).  PBX_CONV_FWD=3 keeps conv_fwd3.
CONV_FWD5 = os.environ.get("PBX_CONV_FWD", "5") == "5"


def conv_dgrad_fin(dh1, s1, st1, T1, BM1, sums1, TS1, g1, gdn, gdw, wtn, wtw, dx, dpn, dpw, dgb, B, L, KS, dil,
                   stream):
    """Conv data gradient with the LayerNorm-1 backward finalize fused in (whole sequences, conv_dgrad4<FIN>):
    dx, both convs' dpre (for the weight gradient) and dgb += the column sums of dS1.  (A persistent form with
    the staging pipelined into the K loop measured no better in the step: profiles/r6/conv_dgrad5_attempts.txt.)"""
    _lib.call("pbx_conv_dgrad4f", dh1.data_ptr(), s1.data_ptr(), st1.data_ptr(), T1, BM1, sums1.data_ptr(),
              TS1, g1.data_ptr(), gdn.data_ptr(), gdw.data_ptr(), wtn.data_ptr(), wtw.data_ptr(),
              dx.data_ptr(), dpn.data_ptr(), dpw.data_ptr(), dgb.data_ptr(), B, L, KS, dil, LN_EPS, stream)


def conv_fwd(x, wpn, wpw, bn, bw, gb, pre_n, pre_w, s1, stats, B, L, KS, dil, stream, xlo: int = 0,
             xhi: int = 0) -> None:
    """``pre_n``/``pre_w``: GELU'(pre-activation) outputs for the backward, or None (no backward).
    ``xlo``/``xhi``: rows of the neighbouring sequence shards around each sample's L rows of ``x``
    (context parallelism, :mod:`..parallel.cp_fused`)."""
    name = "pbx_conv_fwd5x" if (CONV_FWD5 and KS == 9 and dil == 5) else "pbx_conv_fwd3x"
    _lib.call(name, x.data_ptr(), wpn.data_ptr(), wpw.data_ptr(), bn.data_ptr(), bw.data_ptr(),
              gb.data_ptr(), _p(pre_n), _p(pre_w), s1.data_ptr(), stats.data_ptr(), B, L, KS, dil, xlo, xhi, stream)


def conv_dgrad(ds1, pre_n, pre_w, wtn, wtw, dx, dpn, dpw, B, L, KS, dil, stream, ilo: int = 0, ihi: int = 0) -> None:
    """``pre_n``/``pre_w``: the GELU'(pre-activation) images :func:`conv_fwd` stored; ``ilo``/``ihi``:
    neighbouring shards' rows around ``ds1`` / GELU' (context parallelism).  csrc/conv4.hip conv_dgrad4:
    4 waves, each over both convs into one accumulator set."""
    _lib.call("pbx_conv_dgrad4x", ds1.data_ptr(), pre_n.data_ptr(), pre_w.data_ptr(), wtn.data_ptr(),
              wtw.data_ptr(), dx.data_ptr(), dpn.data_ptr(), dpw.data_ptr(), B, L, KS, dil, ilo, ihi, stream)


_DWL_SLAB: Dict[int, torch.Tensor] = {}


def dwl_slab(dev: torch.device) -> Tuple[Optional[int], int]:
    """(pointer, rows) of a per-device [2 x CUs] x (128 x 128 + 128) fp32 scratch slab for the
    local-MLP weight / bias gradient partials of the LayerNorm/MLP backward kernels (one row per
    workgroup, folded by fixed-order column-sum launches; the kernels fall back to float atomics when
    it is too small).  The kernels run on one stream in order, so one slab per device is reused by
    every block."""
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _DWL_SLAB.get(idx)
    rows = 2 * _num_cus(dev)
    if s is None:
        s = torch.empty(rows * (CH * CH + CH), dtype=torch.float32, device=dev)
        _DWL_SLAB[idx] = s
    return s.data_ptr(), rows


def _num_cus(dev: torch.device) -> int:
    return torch.cuda.get_device_properties(dev).multi_processor_count


def pack_conv(w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """fp32 ``[co, ci, KS]`` -> the forward and dgrad bf16 MFMA A-fragment images
    ``[KS][8][4][64 lanes][8]`` (M = co / ci, K = ci / co)."""
    KS = w.shape[2]
    wp = torch.empty((KS, CH, CH), dtype=torch.bfloat16, device=w.device)
    wt = torch.empty_like(wp)
    _lib.call("pbx_pack_conv_frag", w.detach().contiguous().data_ptr(), wp.data_ptr(), wt.data_ptr(), KS,
              _lib.stream_ptr(w.device))
    return wp, wt


def _grad_dst(p: torch.Tensor, shape) -> Tuple[torch.Tensor, bool]:
    """Accumulate straight into the parameter's (arena) .grad when it exists, else a new tensor."""
    g = getattr(p, "grad", None) if getattr(p, "_pbx_arena", False) else None
    if g is not None and g.is_contiguous() and g.dtype == torch.float32 and tuple(g.shape) == tuple(shape):
        return g, True
    return torch.zeros(shape, dtype=torch.float32, device=p.device), False


# the first block's weight gradient is the last kernel of the backward (the main stream only has the
# embedding / input-layer tail left beside it): it takes every CU (the other blocks' take 7/8)
WGRAD_TAIL_FULL = True
# the local-MLP dWl / dbl slab folds run on the weight-gradient stream (False: on the main
# stream right after the LN2 / MLP backward kernel)
LN2_LATE_FOLD = True
# the LN1 backward finalize fused into the conv data gradient (csrc/conv4.hip conv_dgrad4<FIN>): dS1 is
# computed in the staging pass and never stored (False: ln1_finalize + conv_dgrad4); not in the
# deterministic mode (its dgb column sums are float atomics per tile) nor under context parallelism
DGRAD_FIN = True
# the input layer's backward starts beside the first block's conv data gradient (False:
# on the main stream after it)
INPUT_BWD_EARLY = True


# eighths of the CUs the aux-stream conv weight gradient takes (R = 56 chunks at 7 on 256 CUs)
WGRAD_CU_EIGHTHS = 7


def _wgrad(dy0: torch.Tensor, dy1: Optional[torch.Tensor], x: torch.Tensor, KS: int, dil: int, nconv: int,
           B: int, L: int, outs, full_chip: bool = False, xlo: int = 0, xhi: int = 0):
    """outs: [(dw, db)] destinations (accumulated into).  Returns the scratch tensors (the caller keeps
    them alive while the launch may still be running on another stream)."""
    dev = x.device
    ntiles = B * ((L + 127) // 128)
    # csrc/wgrad.hip: one workgroup per CU, R chunks x (nconv x 2) channel halves = 7/8 of the CUs
    # (R = 56 on 256 CUs): the aux-stream weight gradient runs beside the main-stream backward, and
    # leaving it a few CUs measured +2.4 % on the step over R = 64 (R = 48: +1.3 %, 32: -0.4 %)
    R = max(8, (WGRAD_CU_EIGHTHS * _num_cus(dev) // (16 * nconv)) // 8 * 8)
    if full_chip:
        R = max(8, (_num_cus(dev) // (2 * nconv)) // 8 * 8)
    R = min(R, ntiles)
    slab = torch.empty((R, nconv, KS, CH, CH), dtype=torch.float32, device=dev)
    bslab = torch.empty((R, nconv, CH), dtype=torch.float32, device=dev)
    (dw0, db0) = outs[0]
    (dw1, db1) = outs[1] if nconv > 1 else (None, None)
    if xlo or xhi:
        _lib.call("pbx_wgrad2x", dy0.data_ptr(), _p(dy1), x.data_ptr(), slab.data_ptr(), bslab.data_ptr(),
                  dw0.data_ptr(), _p(dw1), db0.data_ptr(), _p(db1), B, L, dil, nconv, R, xlo, xhi, _lib.stream_ptr(dev))
    else:
        _lib.call("pbx_wgrad2", dy0.data_ptr(), _p(dy1), x.data_ptr(), slab.data_ptr(), bslab.data_ptr(),
                  dw0.data_ptr(), _p(dw1), db0.data_ptr(), _p(db1), B, L, dil, nconv, R, _lib.stream_ptr(dev))
    return [slab, bslab]


# the first block's conv weight gradient through the token one-hot (csrc/wgrad.hip wgrad_tok: its input is
# the embedding bf16(E[tok]), so dW = E^T S with S a 32-row one-hot GEMM); False: wgrad2 over the
# 128 embedding channels
WGRAD_TOK = True
# ... and its conv data gradient is folded away: the block input is the embedding, so only
# dE = sum_{tok} (dS1 + conv^T dpre) is needed -- the dS1 part in one pass that also writes dpre
# (pbx_embed_dpre), the conv^T part as bf16(W)-weighted sums of the weight gradient's one-hot S
# (pbx_wgrad_tok).  False: conv data gradient + embedding backward as for any block.
EMBED_FOLD = True
# ... and (reference semantics) its conv gathers emb[tok] in the staging pass: the [B, L, 128] embedding
# output is never written (False: embed_fwd + conv_fwd3)
EMBED_GATHER = True


def wgrad_tok_ok(tok: Optional[torch.Tensor], emb: Optional[torch.Tensor], L: int, KS: int) -> bool:
    return (WGRAD_TOK and tok is not None and emb is not None and KS == 9 and L % 2 == 0
            and emb.shape[0] <= 32 and emb.shape[1] == CH and tok.dtype == torch.int64 and tok.is_contiguous())


def _wgrad_tok(dy0: torch.Tensor, dy1: torch.Tensor, tok: torch.Tensor, emb: torch.Tensor, dil: int, B: int, L: int,
               outs, demb=None):
    """Both conv weight gradients of a block whose input is the embedding bf16(E[tok]); ``outs`` as
    :func:`_wgrad`.  ``demb``: (W_narrow, W_wide, dE) -- also add the convolutions' part of the embedding
    gradient into dE (the block's data gradient is folded away, :data:`EMBED_FOLD`).  Returns the scratch
    tensors (kept alive while the launch may be running)."""
    dev = dy0.device
    V = emb.shape[0]
    R = _lib.lib().pbx_wgrad_tok_rows(B, L)
    slab = torch.empty((R, 2, 9, V, CH), dtype=torch.float32, device=dev)
    S = torch.empty((2, 9, V, CH), dtype=torch.float32, device=dev)
    e = emb.detach().float().contiguous()
    (dw0, db0), (dw1, db1) = outs
    w0 = w1 = dE = dEslab = None
    if demb is not None:
        w0, w1 = (w.detach().float().contiguous() for w in demb[:2])
        dE = demb[2]
        dEslab = torch.empty((2 * CH, V, CH), dtype=torch.float32, device=dev)
    _lib.call("pbx_wgrad_tok", tok.data_ptr(), dy0.data_ptr(), dy1.data_ptr(), e.data_ptr(), slab.data_ptr(),
              S.data_ptr(), dw0.data_ptr(), dw1.data_ptr(), db0.data_ptr(), db1.data_ptr(), B, L, dil, V,
              _p(w0), _p(w1), _p(dE), _p(dEslab), _lib.stream_ptr(dev))
    return [slab, S, e, w0, w1, dEslab]


def embed_fold_bwd(tok, emb, ds1, gdn, gdw, dpn, dpw, wn, ww, stream):
    """First block with its conv data gradient folded away (:data:`EMBED_FOLD`): dE += sum_tok dS1 and
    dpn / dpw = dS1 GELU'(pre) in one pass over dS1 (``pbx_embed_dpre``).  Returns ``((wn, ww, dE),
    direct)``: the ``demb`` argument of :func:`_wgrad_tok` (which adds the convolutions' part of dE) and
    whether dE is the arena gradient itself."""
    B, L = tok.shape
    dE, direct = _grad_dst(emb, emb.shape)
    slab = None
    if fused_deterministic():
        slab = torch.empty((_lib.lib().pbx_embed_bwd_groups(B * L), emb.shape[0], CH), dtype=torch.float32,
                           device=ds1.device)
    _lib.call("pbx_embed_dpre", tok.data_ptr(), ds1.data_ptr(), gdn.data_ptr(), gdw.data_ptr(), dpn.data_ptr(),
              dpw.data_ptr(), dE.data_ptr(), B * L, emb.shape[0], _p(slab), stream)
    return (wn, ww, dE), direct


class LocalBlockFn(torch.autograd.Function):
    """Fused local track of one block (reference semantics)."""

    @staticmethod
    def forward(ctx, x, gb, wn, bn, ww, bw, g1, be1, wl, bl, g2, be2, wv_bf16, dil: int, packed=None,
                tail: bool = False, cp=None, tok=None, emb=None, emb_grad: bool = False):
        """``packed``: (wpn, wtn, wpw, wtw) weight images already built for this step (pack_batch);
        ``tail``: the first block (its backward ends the step: the conv weight gradient gets every CU);
        ``cp``: a :class:`..parallel.cp_fused.CPShard` -- ``x`` is this rank's slice of the sequence, the
        conv reads the neighbours' halo rows and the (L, C) LayerNorm statistics are group-wide;
        ``tok`` / ``emb``: ``x`` is the embedding bf16(emb[tok]) (the first block): the conv weight gradient
        goes through the token one-hot (:func:`_wgrad_tok`); ``emb_grad``: ``x`` carries no autograd
        history and the backward returns ``emb``'s gradient instead of ``x``'s (:data:`EMBED_FOLD`)."""
        params = (wn, bn, ww, bw, g1, be1, wl, bl, g2, be2)
        ctx.cp = cp
        if cp is not None:
            # this shard's rows of the [L, C] LayerNorm affine (contiguous row slices of the parameters)
            g1, be1, g2, be2 = (cp.rows(t) for t in (g1, be1, g2, be2))
        if x is None:
            # the first block, folded (emb_grad): the conv gathers emb[tok] itself (pbx_conv_fwd3t)
            if not (emb_grad and tok is not None and emb is not None and cp is None):
                raise ValueError("x may be None only for the folded first block (emb_grad with tok / emb)")
            B, L = tok.shape
            xt = torch.empty((B, L, CH), dtype=torch.bfloat16, device=tok.device)   # shape template only
        else:
            B, L, C = x.shape
            assert C == CH and x.dtype == torch.bfloat16 and x.is_contiguous()
            xt = x
        NJ = wv_bf16.shape[0]
        if not attn_pool_supported(NJ):
            raise NotImplementedError(f"HIP attention pool: H * value_dim = {NJ} (kernels built for 256 / 512)")
        KS = wn.shape[2]
        dev = xt.device
        stream = _lib.stream_ptr(dev)
        T1 = (L + BM1 - 1) // BM1
        T2 = (L + PB - 1) // PB
        if packed is not None:
            wpn, wtn, wpw, wtw = packed
        else:
            wpn, wtn = pack_conv(wn)
            wpw, wtw = pack_conv(ww)
        wl_b = bf16_of(wl)
        # inference / frozen-encoder forwards keep no backward state: the conv pre-activations, the MLP
        # pre-activation and the pool's GELU' fragments are not written at all
        need_bwd = any(ctx.needs_input_grad)
        pre_n = torch.empty_like(xt) if need_bwd else None
        pre_w = torch.empty_like(xt) if need_bwd else None
        s1 = torch.empty_like(xt)
        st1 = torch.empty((B, T1, 2), dtype=torch.float32, device=dev)
        gb = gb.detach().float().contiguous()
        if x is None:
            x_ext, hlo = None, 0
            emb_b = bf16_of(emb)                  # the optimizer-maintained bf16 mirror: no cast launch
            _lib.call("pbx_conv_fwd3t", tok.data_ptr(), emb_b.data_ptr(), wpn.data_ptr(), wpw.data_ptr(),
                      bn.data_ptr(), bw.data_ptr(), gb.data_ptr(), _p(pre_n), _p(pre_w), s1.data_ptr(),
                      st1.data_ptr(), B, L, KS, dil, stream)
        elif cp is None:
            x_ext, hlo = x, 0
            conv_fwd(x, wpn, wpw, bn, bw, gb, pre_n, pre_w, s1, st1, B, L, KS, dil, stream)
        else:
            x_ext, hlo = cp.halo_rows(x), cp.halo
            conv_fwd(x_ext, wpn, wpw, bn, bw, gb, pre_n, pre_w, s1, st1, B, L, KS, dil, stream, hlo, hlo)
            cp.fix_stats(st1, BM1)
        pre_l = torch.empty_like(xt) if need_bwd else None
        s2 = torch.empty_like(xt)
        st2 = torch.empty((B, T2, 2), dtype=torch.float32, device=dev)
        _lib.call("pbx_ln_linear_fwd", s1.data_ptr(), st1.data_ptr(), T1, BM1, g1.data_ptr(), be1.data_ptr(),
                  wl_b.data_ptr(), bl.data_ptr(), _p(pre_l), s2.data_ptr(), st2.data_ptr(), B, L, LN_EPS, stream)
        if cp is not None:
            cp.fix_stats(st2, PB)
        # LN2 apply + attention pool in one launch (csrc/pool.hip); the backward recomputes GELU' from h2
        h2 = torch.empty_like(xt)
        TV = (L + 31) // 32                     # one vpart row per 32-position tile
        vpart = torch.empty((B, TV, NJ), dtype=torch.float32, device=dev)
        _lib.call("pbx_pool_fwd", s2.data_ptr(), st2.data_ptr(), g2.data_ptr(), be2.data_ptr(), wv_bf16.data_ptr(),
                  h2.data_ptr(), vpart.data_ptr(), B, L, NJ, LN_EPS, stream)
        ctx.save_for_backward(x_ext, pre_n, pre_w, s1, st1, pre_l, s2, st2, h2, wtn, wtw, wl_b, wv_bf16, g1, be1, g2,
                              be2)
        ctx.hlo = hlo
        ctx.tok = (tok, emb) if cp is None and wgrad_tok_ok(tok, emb, L, KS) else None
        ctx.emb_grad = bool(emb_grad)
        if ctx.emb_grad and (ctx.tok is None or (x is not None and x.requires_grad)):
            raise ValueError("emb_grad needs a token-embedding input without autograd history (wgrad_tok_ok)")
        ctx.meta = (B, L, KS, dil, T1, T2, NJ)
        ctx.tail = bool(tail) and WGRAD_TAIL_FULL
        ctx.set_materialize_grads(False)
        ctx.params = params
        return h2, vpart

    @staticmethod
    def backward(ctx, dh2, dvpart):
        streams.wait_ready(dvpart, dh2)         # producers on an aux stream (none by default)
        (x_ext, pre_n, pre_w, s1, st1, pre_l, s2, st2, h2, wtn, wtw, wl_b, wv_bf16, g1, be1, g2,
         be2) = ctx.saved_tensors
        cp, hlo = ctx.cp, ctx.hlo
        x = s1                                  # shape / dtype / device template of the [B, L, C] activations
        B, L, KS, dil, T1, T2, NJ = ctx.meta
        dev = x.device
        stream = _lib.stream_ptr(dev)
        params = ctx.params
        dsts = [_grad_dst(p, p.shape) for p in params]
        (dwn, _), (dbn, _), (dww, _), (dbw, _), (dg1, _), (dbe1, _), (dwl, _), (dbl, _), (dg2, _), (dbe2, _) = dsts
        if cp is not None:
            # this shard's rows of the [L, C] affine gradients (the kernels accumulate into them)
            dg1, dbe1, dg2, dbe2 = (cp.rows(t) for t in (dg1, dbe1, dg2, dbe2))
        dh2 = None if dh2 is None else dh2.to(torch.bfloat16).contiguous()
        # pool backward (csrc/pool.hip): GELU' recomputed from h2, LN2 partials per 32-position tile; the LN2 /
        # LN1 constants come from ln2_consts_kernel inside pbx_ln2_linear_bwd
        TA = (L + 31) // 32
        if dvpart is None:
            dv, dv_tiles = torch.zeros((B, NJ), dtype=torch.float32, device=dev), 1
        elif dvpart.dim() == 3 and (dvpart.shape[1] == 1 or dvpart.stride(1) == 0):
            dv, dv_tiles = dvpart[:, 0, :].float().contiguous(), 1     # one gradient row per sample
        else:
            dv, dv_tiles = dvpart.float().contiguous(), TA
        dh2t = torch.empty_like(x)
        sums2 = torch.empty((B, TA, 2), dtype=torch.float32, device=dev)
        consts = torch.empty((B, 8), dtype=torch.float32, device=dev)
        dgb = torch.empty((B, CH), dtype=torch.float32, device=dev)      # zeroed by the consts writer
        _lib.call("pbx_pool_bwd", h2.data_ptr(), g2.data_ptr(), be2.data_ptr(), _p(dh2), dv.data_ptr(), dv_tiles,
                  wv_bf16.data_ptr(), dh2t.data_ptr(), sums2.data_ptr(), B, L, NJ, stream)
        if cp is not None:
            cp.fix_sums(sums2)
        # LN2 finalize + local MLP backward + LN1 partials + both [L, C] affine gradients
        dh1 = torch.empty_like(x)
        TS1 = (L + 1) // 2                      # LN1 partials per (sample, position pair)
        sums1 = torch.empty((B, TS1, 2), dtype=torch.float32, device=dev)
        det = int(fused_deterministic())
        # the local-MLP weight / bias gradient partials are folded on the weight-gradient stream (only the
        # optimizer and the DP all-reduce read them): a slab of this call's own, the shared one is reused
        # by the next block's kernel while the fold may still be queued
        late_fold = LN2_LATE_FOLD and streams.ENABLED and dev.type == "cuda" and dsts[6][1] and dsts[7][1]
        if late_fold:
            rows = _lib.lib().pbx_ln2_bwd_slab_rows(B, L, det)
            fslab = torch.empty(rows * (CH * CH + CH), dtype=torch.float32, device=dev)
            slab_args = (fslab.data_ptr(), rows)
        else:
            slab_args = dwl_slab(dev)
        _lib.call("pbx_ln2_linear_bwd", dh2t.data_ptr(), s2.data_ptr(), st2.data_ptr(), sums2.data_ptr(), TA,
                  g2.data_ptr(), pre_l.data_ptr(), s1.data_ptr(), st1.data_ptr(), T1, BM1, g1.data_ptr(),
                  be1.data_ptr(), wl_b.data_ptr(), consts.data_ptr(), dh1.data_ptr(), sums1.data_ptr(),
                  dg2.data_ptr(), dbe2.data_ptr(), dg1.data_ptr(), dbe1.data_ptr(), dwl.data_ptr(), dbl.data_ptr(),
                  dgb.data_ptr(), B, L, LN_EPS, *slab_args, det, int(not late_fold), 0, stream)
        if late_fold:
            def fold(slab=fslab, rows=rows, dwl=dwl, dbl=dbl):
                st = _lib.stream_ptr(dev)
                _lib.call("pbx_colsum_add2", slab.data_ptr(), CH * CH, dwl.data_ptr(), slab[rows * CH * CH:].data_ptr(),
                          CH, dbl.data_ptr(), rows, st)
            streams.launch(dev, fold, keep=[fslab], name="wgrad")
        dx = None if ctx.emb_grad else torch.empty_like(x)
        dpn = torch.empty_like(x)
        dpw = torch.empty_like(x)
        if cp is not None:
            cp.fix_sums(sums1)
        # the LN1 finalize fused into the conv data gradient (DGRAD_FIN; its dgb is final only after it)
        fin = (DGRAD_FIN and cp is None and not ctx.emb_grad and KS == 9 and dev.type == "cuda"
               and not fused_deterministic())

        def dgb_ready():
            if ctx.tail and INPUT_BWD_EARLY and streams.ENABLED and dev.type == "cuda":
                # first block: the input layer's backward (the last autograd node but one) needs only dgb
                # and the global-track gradient, both final here -- it runs on the "ann" stream beside this
                # conv data gradient, so its 18 MB weight-gradient bucket is ready ~0.2 ms earlier for the
                # DP all-reduce (ops/global_track.py InputLayerFn.backward)
                streams.fork(dev, "ann")

        if not fin:
            # LN1 finalize (ds1) + gradient of the broadcast global->local vector
            ds1 = torch.empty_like(x)
            _lib.call("pbx_ln1_finalize", dh1.data_ptr(), s1.data_ptr(), st1.data_ptr(), T1, BM1, sums1.data_ptr(),
                      TS1, g1.data_ptr(), ds1.data_ptr(), dgb.data_ptr(), B, L, LN_EPS, int(fused_deterministic()),
                      stream)
            if cp is not None:
                cp.all_reduce_(dgb)             # gb is replicated: its gradient sums every shard's positions
            dgb_ready()
        demb = None
        if fin:
            conv_dgrad_fin(dh1, s1, st1, T1, BM1, sums1, TS1, g1, pre_n, pre_w, wtn, wtw, dx, dpn, dpw, dgb, B, L,
                           KS, dil, stream)
            dgb_ready()
        elif ctx.emb_grad:
            # first block, folded: no conv data gradient (the conv part of dE comes with the weight gradient)
            demb, dE_direct = embed_fold_bwd(*ctx.tok, ds1, pre_n, pre_w, dpn, dpw, params[0], params[2], stream)
            dE = demb[2]
        elif cp is None:
            conv_dgrad(ds1, pre_n, pre_w, wtn, wtw, dx, dpn, dpw, B, L, KS, dil, stream)
        else:
            # the transposed conv reads dpre = ds1 GELU' of the neighbours' edge rows too
            conv_dgrad(*cp.halo_rows_many(ds1, pre_n, pre_w), wtn, wtw, dx, dpn, dpw, B, L,
                       KS, dil, stream, hlo, hlo)
        if ctx.tok is not None:
            tok, emb = ctx.tok
            wg = lambda: _wgrad_tok(dpn, dpw, tok, emb, dil, B, L, [(dwn, dbn), (dww, dbw)], demb)   # noqa: E731
            keep = [dpn, dpw, tok] + ([demb[2]] if demb is not None else [])
        else:
            wg = lambda: _wgrad(dpn, dpw, x_ext, KS, dil, 2, B, L, [(dwn, dbn), (dww, dbw)],   # noqa: E731
                                ctx.tail and streams.ENABLED, hlo, hlo)
            keep = [dpn, dpw, x_ext]
        direct = [p for p, (_, d) in zip(params, dsts) if d]
        if demb is not None and dE_direct:
            direct.append(ctx.tok[1])
        if all(dsts[i][1] for i in (0, 1, 2, 3)) and (demb is None or dE_direct) and streams.ENABLED:
            # the weight gradient goes to the aux stream: off the critical path, only the optimizer
            # and the DP all-reduce read it (its inputs stay referenced until the join)
            streams.launch(dev, wg, keep=keep, name="wgrad")
        else:
            wg()
        if direct:
            notify_grads_ready(direct)
        pgrads = [None if d else g for (g, d) in dsts]
        gemb = dE if demb is not None and not dE_direct else None
        return (dx, dgb, *pgrads, None, None, None, None, None, None, gemb, None)


def embed_tokens(tokens: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """bf16(weight[tokens]) without autograd history (the folded first block returns the weight's
    gradient itself, :data:`EMBED_FOLD`)."""
    B, L = tokens.shape
    tok = tokens.contiguous()
    out = torch.empty((B, L, weight.shape[1]), dtype=torch.bfloat16, device=tokens.device)
    _lib.call("pbx_embed_fwd", tok.data_ptr(), weight.detach().contiguous().data_ptr(), out.data_ptr(), B * L,
              _lib.stream_ptr(tokens.device))
    return out


class EmbedFn(torch.autograd.Function):
    """Token embedding gather to bf16 (reference ``modules.py:249-253,300``); backward is a 26-row
    segmented sum instead of torch's sort-based ``embedding_dense_backward``."""

    @staticmethod
    def forward(ctx, tokens, weight):
        B, L = tokens.shape
        V, C = weight.shape
        assert C == CH and V <= 32
        tok = tokens.contiguous()
        out = torch.empty((B, L, C), dtype=torch.bfloat16, device=tokens.device)
        _lib.call("pbx_embed_fwd", tok.data_ptr(), weight.detach().contiguous().data_ptr(), out.data_ptr(), B * L,
                  _lib.stream_ptr(tokens.device))
        ctx.save_for_backward(tok)
        ctx.V = V
        return out

    @staticmethod
    def backward(ctx, dout):
        (tok,) = ctx.saved_tensors
        dE = torch.zeros((ctx.V, CH), dtype=torch.float32, device=tok.device)
        d = dout.to(torch.bfloat16).contiguous()
        slab = None
        if fused_deterministic():
            g = _lib.lib().pbx_embed_bwd_groups(tok.numel())
            slab = torch.empty((g, ctx.V, CH), dtype=torch.float32, device=tok.device)
        _lib.call("pbx_embed_bwd", tok.data_ptr(), d.data_ptr(), dE.data_ptr(), tok.numel(), ctx.V, _lib.ptr(slab),
                  _lib.stream_ptr(tok.device))
        return None, dE


def _wv_bf16(att) -> torch.Tensor:
    """bf16 [H*vd, C] copy of the stacked value weights.  In reference semantics the heads are
    untrained buffers, so the copy is cached and only rebuilt when Wv changes."""
    Wv = att.Wv
    if isinstance(Wv, torch.nn.Parameter) and Wv.requires_grad:
        return att.value_weight_cat().t().to(torch.bfloat16).contiguous()
    key = (Wv.data_ptr(), Wv._version, Wv.device)
    cached = getattr(att, "_pbx_wv_cache", None)
    if cached is None or cached[0] != key:
        cached = (key, att.value_weight_cat().t().to(torch.bfloat16).contiguous())
        att._pbx_wv_cache = cached
    return cached[1]


def conv_images(wn: torch.Tensor, ww: torch.Tensor):
    """Output buffers of one block's conv weight images and their pack_batch items."""
    KS = wn.shape[2]
    imgs = tuple(torch.empty((KS, CH, CH), dtype=torch.bfloat16, device=wn.device) for _ in range(4))
    return imgs, [(0, wn.detach(), imgs[0], imgs[1], KS, 0), (0, ww.detach(), imgs[2], imgs[3], KS, 0)]


def local_block(x: torch.Tensor, gb: torch.Tensor, blk, packed=None, tail: bool = False,
                cp=None, tok=None, emb=None, emb_grad: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """Run the fused local track of ``blk`` (a ``ProteinBERTBlock``); ``tail``: it is the first block;
    ``cp``: context-parallel shard (:class:`..parallel.cp_fused.CPShard`); ``tok`` / ``emb``: ``x`` is
    the token embedding bf16(emb[tok]); ``emb_grad``: the backward returns ``emb``'s gradient (``x``
    from :func:`embed_tokens`, no autograd history)."""
    att = blk.global_attention_layer
    wv = _wv_bf16(att)                                                       # [H*vd, C]
    nc = blk.local_narrow_conv_layer[0]
    wc = blk.local_wide_conv_layer[0]
    return LocalBlockFn.apply(x, gb, nc.weight, nc.bias, wc.weight, wc.bias, blk.local_norm_1.weight,
                              blk.local_norm_1.bias, blk.local_linear_layer[0].weight, blk.local_linear_layer[0].bias,
                              blk.local_norm_2.weight, blk.local_norm_2.bias, wv, blk.wide_conv_dilation, packed,
                              tail, cp, tok, emb, emb_grad)
