"""Autograd wrappers of the fused CDNA4 local-track kernels (``csrc/conv.hip``, ``csrc/ln.hip``).

One :class:`LocalBlockFn` call is the whole local track of one ``ProteinBERTBlock`` in reference
semantics (reference ``ProteinBERT/modules.py:201-219``)::

    s1 = x + GELU(conv_d1(x)) + GELU(conv_d5(x)) + gb       (conv_fwd: 1 launch)
    h1 = LN_(L,C)(s1); s2 = h1 + GELU(h1 Wl^T + bl)           (ln_linear_fwd: 1 launch)
    h2 = LN_(L,C)(s2); vpart = sum_tile GELU(h2 Wv_cat^T)     (ln_attn_fwd: 1 launch)

and its backward is 9 launches (attention/LN2, LN2 affine, LN2+MLP, MLP wgrad, LN1 affine+finalize,
conv dgrad, conv wgrad).  Activations are bf16 ``[B, L, 128]`` channels-last; parameters stay fp32
masters and are packed to bf16 kernel layouts once per forward.  The global track (``[B, 512]``
vectors) stays in PyTorch: it is ~0.1 % of the FLOPs.

Every op raises if the HIP library is missing — there is no silent eager fallback on a GPU.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional, Tuple

import torch

from . import _lib, streams
from ..train.arena import notify_grads_ready
from .global_track import bf16_of

_P, _I, _F, _L = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_long

_lib.register("pbx_conv_fwd", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P])
_lib.register("pbx_conv_dgrad", [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P])
_lib.register("pbx_conv_fwd3", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P])
_lib.register("pbx_conv_fwd3x", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P])
_lib.register("pbx_ln_linear_fwdx", [_P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _F, _P])
_lib.register("pbx_ln1_finalizex", [_P, _P, _P, _I, _I, _P, _I, _P, _P, _P, _P, _P, _I, _I, _F, _P])
_lib.register("pbx_conv_dgrad3", [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P])
_lib.register("pbx_conv_dgrad3_ln", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P])
_lib.register("pbx_ln1_consts", [_P, _I, _I, _P, _I, _P, _P, _I, _I, _F, _P])
_lib.register("pbx_pack_conv_frag", [_P, _P, _P, _I, _P])
_lib.register("pbx_wgrad", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P])
_lib.register("pbx_wgrad2", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P])
_lib.register("pbx_pack_conv", [_P, _P, _P, _I, _P])
_lib.register("pbx_ln_linear_fwd", [_P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _I, _I, _F, _P])
_lib.register("pbx_ln_attn_fwd", [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _F, _P])
_lib.register("pbx_attn_bwd", [_P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _I, _I, _I, _I, _F, _P])
_lib.register("pbx_ln_attn_fwd2", [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _F, _P])
_lib.register("pbx_attn_bwd2", [_P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _I, _I, _I, _F, _P])
_lib.register("pbx_ln2_linear_bwd", [_P, _P, _P, _P, _I, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P,
                                     _P, _P, _P, _P, _P, _I, _I, _F, _P])  # ..wl, consts, dh1, sums1, dg2..dbl, dgb
_lib.register("pbx_ln2_linear_bwd2", [_P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P,
                                      _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _F, _I, _P, _I, _P])
_lib.register("pbx_ln1_finalize", [_P, _P, _P, _I, _I, _P, _I, _P, _P, _P, _I, _I, _F, _P])
_lib.register("pbx_embed_fwd", [_P, _P, _P, _L, _P])
_lib.register("pbx_embed_bwd", [_P, _P, _P, _L, _I, _P])

CH = 128          # kernels are specialised for local_dim = 128
PB = 32           # positions per workgroup of the position-major LayerNorm kernels
LN_EPS = 1e-5     # nn.LayerNorm default (reference modules.py:148-164)


# conv kernel form: "v3" (csrc/conv2.hip: weights streamed from L2 as packed MFMA fragments,
# 128-position tiles, two workgroups per CU) or "v1" (csrc/conv.hip: weights staged through an LDS
# ring, 256/128-position tiles, one workgroup per CU); PBX_CONV=v1 selects the latter.
CONV_IMPL = os.environ.get("PBX_CONV", "v3")
# conv weight-gradient form (k = 9): "v2" (csrc/wgrad.hip: LDS-DMA double buffer, 64 output channels
# per workgroup, one workgroup per CU) or "v1" (csrc/conv.hip wgrad_kernel); PBX_WGRAD=v1 selects v1.
WGRAD_IMPL = os.environ.get("PBX_WGRAD", "v2")


# attention-pool form: "v2" (the forward stores GELU' as bf16 MFMA fragments, the backward streams
# them: no recompute GEMM, no transcendental in the backward) or "v1" (backward recomputes h2 Wv and
# GELU'); PBX_ATTN_POOL=v1 selects the latter.  v2 needs NJ = H*VD in (256, 512).
ATTN_POOL = os.environ.get("PBX_ATTN_POOL", "v2")


# pool-v2 forward launch: waves per workgroup | GELU pairs per interleaved core call << 4
# (12: 32-position items, three waves per SIMD, vpart rows per 32 positions; measured equal to slightly
# slower than 8 on the B=512 L=512 step, profiles/r2_v8_pool_32pos_ab.txt: more waves do not help a
# kernel whose SIMDs are already issue-bound on the GELU / GELU' VALU work)
ATTN_FWD2_CFG = int(os.environ.get("PBX_ATTN_FWD2", "8"), 0)


def attn_pool_v2(NJ: int) -> bool:
    return ATTN_POOL == "v2" and NJ in (256, 512)


# v3 forward tile: 128 positions (two workgroups per CU; measured faster in the full step than 256,
# one workgroup per CU with each streamed weight fragment feeding 8 MFMAs); PBX_CONV_TILE=256 selects it
CONV3_TILE = int(os.environ.get("PBX_CONV_TILE", "128"))
# local-MLP pre-activation: "recompute" (the LN2/MLP backward recomputes h1 Wl^T + bl on MFMA, the
# forward stores nothing) or "store" (forward writes it as a bf16 [B, L, 128] tensor)
PRE_L = os.environ.get("PBX_PRE_L", "store")
# workgroups per CU the LN2/MLP backward grid aims at (0: one)
LN2_WG_PER_CU = int(os.environ.get("PBX_LN2_WGCU", "0"))
# "late gb": the conv forward stores s1 WITHOUT the broadcast global->local vector gb (plus per-tile
# channel sums), the LN1 consumers add it and correct the statistics exactly; the conv then no longer
# waits for the previous block's global track, which runs beside it on an aux stream.  Measured 1-2 %
# SLOWER on the B=512 L=512 step (same-box A/B, high- or normal-priority aux stream: the 32 global-track
# workgroups find no CU with free LDS beside the convolution's), so it is opt-in.
LATE_GB = os.environ.get("PBX_LATE_GB", "0") == "1"
# LayerNorm-1 backward inside the conv data gradient (csrc/conv2.hip conv_dgrad3_kernel<true>): the
# kernel reads dh1, s1 and g1 and builds ds1 itself (halo rows included) instead of a separate finalize
# pass writing ds1 for it.  Measured 1.5-3 % SLOWER on the B=512 L=512 step (same-box A/B, 3 rounds,
# profiles/r2_v8_ln1_fuse_ab.txt): the data-gradient prologue is load-latency bound and now carries
# 2.5x the bytes per round trip, which costs more than the 40 us finalize pass it replaces.  Opt-in.
LN1_FUSE = os.environ.get("PBX_LN1_FUSE", "0") == "1"


def ln1_fused(gb_late) -> bool:
    """LN1 backward fused into the conv data gradient: v3 convs, s1 holding the broadcast vector."""
    return LN1_FUSE and CONV_IMPL == "v3" and gb_late is None


def late_gb_enabled() -> bool:
    return LATE_GB and CONV_IMPL == "v3"


def conv_tile(L: int) -> int:
    """Positions per forward conv workgroup (= the tile of the LayerNorm-1 partials)."""
    if CONV_IMPL == "v3":
        return CONV3_TILE if L >= CONV3_TILE else 128
    return 256 if L >= 256 else 128


def conv_fwd(x, wpn, wpw, bn, bw, gb, pre_n, pre_w, s1, stats, B, L, KS, dil, BM, stream, colsum=None) -> None:
    """``gb`` None (v3 only): s1 without the broadcast vector, ``colsum`` [B, T, 128] its tile channel sums;
    ``pre_n``/``pre_w`` None (v3 only): the pre-activations are not stored (no backward)."""
    if CONV_IMPL == "v3":
        _lib.call("pbx_conv_fwd3x", x.data_ptr(), wpn.data_ptr(), wpw.data_ptr(), bn.data_ptr(), bw.data_ptr(),
                  _p(gb), _p(pre_n), _p(pre_w), s1.data_ptr(), stats.data_ptr(), _p(colsum), B, L, KS,
                  dil, BM, stream)
    else:
        if pre_n is None:
            pre_n, pre_w = torch.empty_like(x), torch.empty_like(x)
        _lib.call("pbx_conv_fwd", x.data_ptr(), wpn.data_ptr(), wpw.data_ptr(), bn.data_ptr(), bw.data_ptr(),
                  gb.data_ptr(), pre_n.data_ptr(), pre_w.data_ptr(), s1.data_ptr(), stats.data_ptr(), B, L, KS, dil,
                  BM, stream)


def conv_dgrad(ds1, pre_n, pre_w, wtn, wtw, dx, dpn, dpw, B, L, KS, dil, BM, stream) -> None:
    if CONV_IMPL == "v3":
        _lib.call("pbx_conv_dgrad3", ds1.data_ptr(), pre_n.data_ptr(), pre_w.data_ptr(), wtn.data_ptr(),
                  wtw.data_ptr(), dx.data_ptr(), dpn.data_ptr(), dpw.data_ptr(), B, L, KS, dil, stream)
    else:
        _lib.call("pbx_conv_dgrad", ds1.data_ptr(), pre_n.data_ptr(), pre_w.data_ptr(), wtn.data_ptr(),
                  wtw.data_ptr(), dx.data_ptr(), dpn.data_ptr(), dpw.data_ptr(), B, L, KS, dil, BM, stream)


def attn_fwd_waves(L: int) -> int:
    """ln_attn_fwd workgroup: 8 independent waves (work items are 64-position wave tiles)."""
    return 8


def attn_bwd_waves(L: int) -> int:
    """attn_bwd workgroup: 8 independent waves (work items are 32-position wave tiles);
    PBX_ATTN_BWD_WAVES=4 selects the one-wave-per-SIMD (512-register) build."""
    return int(os.environ.get("PBX_ATTN_BWD_WAVES", 8))


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


_DWL_SLAB: Dict[int, torch.Tensor] = {}
DWL_SLAB = os.environ.get("PBX_DWL_SLAB", "1") == "1"


def dwl_slab(dev: torch.device) -> Tuple[Optional[int], int]:
    """(pointer, rows) of a per-device [2 x CUs, 128, 128] fp32 scratch slab for the local-MLP weight
    gradient partials of the LayerNorm/MLP backward kernels (one row per workgroup, folded by one
    column-sum launch; the kernels fall back to float atomics when it is absent or too small).  The
    kernels run on one stream in order, so one slab per device is reused by every block."""
    if not DWL_SLAB:
        return None, 0
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _DWL_SLAB.get(idx)
    if s is None:
        s = torch.empty((2 * _num_cus(dev), CH, CH), dtype=torch.float32, device=dev)
        _DWL_SLAB[idx] = s
    return s.data_ptr(), s.shape[0]


def _num_cus(dev: torch.device) -> int:
    return torch.cuda.get_device_properties(dev).multi_processor_count


def pack_conv(w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """fp32 ``[co, ci, KS]`` -> the forward and dgrad bf16 weight images of the selected conv form:
    v3: MFMA A-fragment images ``[KS][8][4][64 lanes][8]`` (M = co / ci, K = ci / co);
    v1: ``WP[KS][co][ci]`` and ``WT[KS][ci][co]``."""
    KS = w.shape[2]
    wp = torch.empty((KS, CH, CH), dtype=torch.bfloat16, device=w.device)
    wt = torch.empty_like(wp)
    fn = "pbx_pack_conv_frag" if CONV_IMPL == "v3" else "pbx_pack_conv"
    _lib.call(fn, w.detach().contiguous().data_ptr(), wp.data_ptr(), wt.data_ptr(), KS, _lib.stream_ptr(w.device))
    return wp, wt


def _grad_dst(p: torch.Tensor, shape) -> Tuple[torch.Tensor, bool]:
    """Accumulate straight into the parameter's (arena) .grad when it exists, else a new tensor."""
    g = getattr(p, "grad", None) if getattr(p, "_pbx_arena", False) else None
    if g is not None and g.is_contiguous() and g.dtype == torch.float32 and tuple(g.shape) == tuple(shape):
        return g, True
    return torch.zeros(shape, dtype=torch.float32, device=p.device), False


def _wgrad(dy0: torch.Tensor, dy1: Optional[torch.Tensor], x: torch.Tensor, KS: int, dil: int, nconv: int,
           B: int, L: int, outs):
    """outs: [(dw, db)] destinations (accumulated into).  Returns the scratch tensors (the caller keeps
    them alive while the launch may still be running on another stream)."""
    dev = x.device
    ntiles = B * ((L + 127) // 128)
    if KS == 9 and WGRAD_IMPL == "v2":
        # csrc/wgrad.hip: one workgroup per CU, R chunks x (nconv x 2) channel halves = 7/8 of the CUs
        # (R = 56 on 256 CUs): the aux-stream weight gradient runs beside the main-stream backward, and
        # leaving it a few CUs measured +2.4 % on the step over R = 64 (R = 48: +1.3 %, 32: -0.4 %)
        R = int(os.environ.get("PBX_WGRAD_R", 0)) or max(8, (7 * _num_cus(dev) // (16 * nconv)) // 8 * 8)
        R = min(R, ntiles)
        slab = torch.empty((R, nconv, KS, CH, CH), dtype=torch.float32, device=dev)
        bslab = torch.empty((R, nconv, CH), dtype=torch.float32, device=dev)
        (dw0, db0) = outs[0]
        (dw1, db1) = outs[1] if nconv > 1 else (None, None)
        _lib.call("pbx_wgrad2", dy0.data_ptr(), _p(dy1), x.data_ptr(), slab.data_ptr(), bslab.data_ptr(),
                  dw0.data_ptr(), _p(dw1), db0.data_ptr(), _p(db1), B, L, dil, nconv, R, _lib.stream_ptr(dev))
        return [slab, bslab]
    # position chunks: ~3/8 of a CU's worth of workgroups per conv type (R = 48 on 256 CUs), a
    # multiple of 8 for the XCD-aware mapping; measured best with the wgrad on the aux stream, where
    # it shares the chip with the main-stream backward kernels (R = 32/40/56/64/128 are slower)
    R = int(os.environ.get("PBX_WGRAD_R", 0)) or max(8, (3 * _num_cus(dev) // (8 * nconv)) // 8 * 8)
    R = min(R, ntiles)
    slab = torch.empty((R, nconv, KS, CH, CH), dtype=torch.float32, device=dev)
    bslab = torch.empty((R, nconv, CH), dtype=torch.float32, device=dev)
    (dw0, db0) = outs[0]
    (dw1, db1) = outs[1] if nconv > 1 else (None, None)
    _lib.call("pbx_wgrad", dy0.data_ptr(), _p(dy1), x.data_ptr(), slab.data_ptr(), bslab.data_ptr(),
              dw0.data_ptr(), _p(dw1), db0.data_ptr(), _p(db1), B, L, KS, dil, nconv, R, 1, _lib.stream_ptr(dev))
    return [slab, bslab]


class LocalBlockFn(torch.autograd.Function):
    """Fused local track of one block (reference semantics)."""

    @staticmethod
    def forward(ctx, x, gb, wn, bn, ww, bw, g1, be1, wl, bl, g2, be2, wv_bf16, dil: int, packed=None):
        """``packed``: (wpn, wtn, wpw, wtw) weight images already built for this step (pack_batch)."""
        params = (wn, bn, ww, bw, g1, be1, wl, bl, g2, be2)
        B, L, C = x.shape
        assert C == CH and x.dtype == torch.bfloat16 and x.is_contiguous()
        KS = wn.shape[2]
        dev = x.device
        stream = _lib.stream_ptr(dev)
        BM1 = conv_tile(L)
        T1 = (L + BM1 - 1) // BM1
        T2 = (L + PB - 1) // PB
        if packed is not None:
            wpn, wtn, wpw, wtw = packed
        else:
            wpn, wtn = pack_conv(wn)
            wpw, wtw = pack_conv(ww)
        wl_b = bf16_of(wl)
        late = late_gb_enabled()
        # inference / frozen-encoder forwards keep no backward state: the conv pre-activations, the MLP
        # pre-activation and the pool's GELU' fragments are not written at all
        need_bwd = any(ctx.needs_input_grad)
        pre_n = torch.empty_like(x) if need_bwd else None
        pre_w = torch.empty_like(x) if need_bwd else None
        s1 = torch.empty_like(x)
        st1 = torch.empty((B, T1, 2), dtype=torch.float32, device=dev)
        cs1 = st1f = None
        if late:
            # s1 without gb: the convolution does not wait for the global track producing gb
            cs1 = torch.empty((B, T1, CH), dtype=torch.float32, device=dev)
            st1f = torch.empty((B, 2), dtype=torch.float32, device=dev)
            conv_fwd(x, wpn, wpw, bn, bw, None, pre_n, pre_w, s1, st1, B, L, KS, dil, BM1, stream, cs1)
            streams.wait_ready(gb)
            gb = gb.detach().float().contiguous()
        else:
            gb = gb.detach().float().contiguous()
            conv_fwd(x, wpn, wpw, bn, bw, gb, pre_n, pre_w, s1, st1, B, L, KS, dil, BM1, stream)
        pre_l = torch.empty_like(x) if PRE_L == "store" and need_bwd else None
        s2 = torch.empty_like(x)
        st2 = torch.empty((B, T2, 2), dtype=torch.float32, device=dev)
        _lib.call("pbx_ln_linear_fwdx", s1.data_ptr(), st1.data_ptr(), T1, BM1, g1.data_ptr(), be1.data_ptr(),
                  wl_b.data_ptr(), bl.data_ptr(), _p(pre_l), s2.data_ptr(), st2.data_ptr(), _p(gb if late else None),
                  _p(cs1), _p(st1f), B, L, LN_EPS, stream)
        NJ = wv_bf16.shape[0]
        nwf = attn_fwd_waves(L)
        TV = (L + 63) // 64                     # one vpart row per 64-position wave tile
        # the GELU' fragments only serve a backward pass: inference / frozen-encoder forwards skip them
        ctx.pool_v2 = attn_pool_v2(NJ) and need_bwd
        BMV = 64                                # positions per vpart row
        if ctx.pool_v2 and ATTN_FWD2_CFG & 15 == 12:
            BMV = 32                            # 32-position work items: one vpart row each
        TVR = (L + 63) // 64 * (64 // BMV)
        h2 = torch.empty_like(x)
        vpart = torch.empty((B, TVR, NJ), dtype=torch.float32, device=dev)
        if ctx.pool_v2:
            # GELU' of the pool as bf16 backward-operand fragments: [B][2 ceil(L/64) tiles of 32][NJ * 32]
            gfrag = torch.empty((B, 2 * TV, NJ * 32), dtype=torch.bfloat16, device=dev)
            _lib.call("pbx_ln_attn_fwd2", s2.data_ptr(), st2.data_ptr(), g2.data_ptr(), be2.data_ptr(),
                      wv_bf16.data_ptr(), h2.data_ptr(), vpart.data_ptr(), gfrag.data_ptr(), B, L, NJ,
                      ATTN_FWD2_CFG, LN_EPS, stream)
            hsave = gfrag
        else:
            _lib.call("pbx_ln_attn_fwd", s2.data_ptr(), st2.data_ptr(), g2.data_ptr(), be2.data_ptr(),
                      wv_bf16.data_ptr(), h2.data_ptr(), vpart.data_ptr(), B, L, NJ, nwf, LN_EPS, stream)
            hsave = h2
        ctx.save_for_backward(x, pre_n, pre_w, s1, st1, pre_l if pre_l is not None else bl, s2, st2, hsave, wtn,
                              wtw, wl_b, wv_bf16, g1, be1, g2, gb if late else None, st1f)
        ctx.pre_l_stored = pre_l is not None
        ctx.meta = (B, L, KS, dil, BM1, T1, T2, NJ, BMV)
        ctx.set_materialize_grads(False)
        ctx.params = params
        return h2, vpart

    @staticmethod
    def backward(ctx, dh2, dvpart):
        streams.wait_ready(dvpart)           # produced by the global-track backward on its aux stream
        # hs: the GELU' fragments (v2 pool) or h2 (v1 pool, recomputed projection)
        (x, pre_n, pre_w, s1, st1, pre_l, s2, st2, hs, wtn, wtw, wl_b, wv_bf16, g1, be1, g2, gb_late,
         st1f) = ctx.saved_tensors
        B, L, KS, dil, BM1, T1, T2, NJ, BMV = ctx.meta
        dev = x.device
        stream = _lib.stream_ptr(dev)
        params = ctx.params
        dsts = [_grad_dst(p, p.shape) for p in params]
        (dwn, _), (dbn, _), (dww, _), (dbw, _), (dg1, _), (dbe1, _), (dwl, _), (dbl, _), (dg2, _), (dbe2, _) = dsts
        dh2 = None if dh2 is None else dh2.to(torch.bfloat16).contiguous()
        TV = (L + BMV - 1) // BMV
        if dvpart is None:
            dvpart = torch.zeros((B, TV, NJ), dtype=torch.float32, device=dev)
        if dvpart.dim() == 3 and dvpart.stride(1) == 0:
            # same gradient for every forward tile (it comes from sum_t vpart): one row per sample
            dvpart = dvpart[:, 0, :].float().contiguous()
            BMV = (L + 31) // 32 * 32
        elif dvpart.shape[1] != TV:
            dvpart = dvpart[:, :TV]             # 32-position items: a trailing all-padding tile row
        dvpart = dvpart.float().contiguous()
        # attention pool + LN2 partials
        nwb = attn_bwd_waves(L)
        TA = (L + 31) // 32                      # LN2 partials per 32-position wave tile
        dh2t = torch.empty_like(x)
        sums2 = torch.empty((B, TA, 2), dtype=torch.float32, device=dev)
        if ctx.pool_v2:
            _lib.call("pbx_attn_bwd2", hs.data_ptr(), s2.data_ptr(), st2.data_ptr(), g2.data_ptr(), _p(dh2),
                      dvpart.data_ptr(), BMV, wv_bf16.data_ptr(), dh2t.data_ptr(), sums2.data_ptr(), B, L, NJ,
                      LN_EPS, stream)
        else:
            _lib.call("pbx_attn_bwd", hs.data_ptr(), s2.data_ptr(), st2.data_ptr(), g2.data_ptr(), _p(dh2),
                      dvpart.data_ptr(), BMV, wv_bf16.data_ptr(), dh2t.data_ptr(), sums2.data_ptr(), B, L, NJ, nwb,
                      LN_EPS, stream)
        # LN2 finalize + local MLP backward + LN1 partials + both [L, C] affine gradients
        dh1 = torch.empty_like(x)
        TS1 = (L + 1) // 2                      # LN1 partials per (sample, position pair)
        sums1 = torch.empty((B, TS1, 2), dtype=torch.float32, device=dev)
        consts = torch.empty((B, 8), dtype=torch.float32, device=dev)
        dgb = torch.empty((B, CH), dtype=torch.float32, device=dev)      # zeroed by the consts kernel
        # pre_l slot: the stored pre-activation, or the MLP bias it is recomputed with
        pre_ptr, bl_ptr = (pre_l.data_ptr(), None) if ctx.pre_l_stored else (None, pre_l.data_ptr())
        _lib.call("pbx_ln2_linear_bwd2", dh2t.data_ptr(), s2.data_ptr(), st2.data_ptr(), sums2.data_ptr(), TA,
                  g2.data_ptr(), pre_ptr, bl_ptr, s1.data_ptr(), st1.data_ptr(), T1, BM1, g1.data_ptr(),
                  be1.data_ptr(), wl_b.data_ptr(), consts.data_ptr(), dh1.data_ptr(), sums1.data_ptr(),
                  dg2.data_ptr(), dbe2.data_ptr(), dg1.data_ptr(), dbe1.data_ptr(), dwl.data_ptr(), dbl.data_ptr(),
                  dgb.data_ptr(), _p(gb_late), _p(st1f), B, L, LN_EPS, LN2_WG_PER_CU, *dwl_slab(dev), stream)
        dx = torch.empty_like(x)
        dpn = torch.empty_like(x)
        dpw = torch.empty_like(x)
        if ln1_fused(gb_late):
            # LN1 backward (ds1) + gradient of the broadcast global->local vector inside the conv data
            # gradient; only the per-sample constants are a separate (one wave per sample) launch
            c1 = torch.empty((B, 4), dtype=torch.float32, device=dev)
            _lib.call("pbx_ln1_consts", st1.data_ptr(), T1, BM1, sums1.data_ptr(), TS1, _p(st1f), c1.data_ptr(),
                      B, L, LN_EPS, stream)
            _lib.call("pbx_conv_dgrad3_ln", dh1.data_ptr(), s1.data_ptr(), g1.data_ptr(), c1.data_ptr(),
                      dgb.data_ptr(), pre_n.data_ptr(), pre_w.data_ptr(), wtn.data_ptr(), wtw.data_ptr(),
                      dx.data_ptr(), dpn.data_ptr(), dpw.data_ptr(), B, L, KS, dil, stream)
            if streams.GLOBAL_ENABLED:
                streams.fork(dev, "global")
        else:
            # LN1 finalize (ds1) + gradient of the broadcast global->local vector
            ds1 = torch.empty_like(x)
            _lib.call("pbx_ln1_finalizex", dh1.data_ptr(), s1.data_ptr(), st1.data_ptr(), T1, BM1,
                      sums1.data_ptr(), TS1, g1.data_ptr(), ds1.data_ptr(), dgb.data_ptr(), _p(gb_late), _p(st1f),
                      B, L, LN_EPS, stream)
            if streams.GLOBAL_ENABLED:
                # the previous block's global-track backward (next autograd node, aux stream) needs only
                # dgb: let it start here, beside the conv data gradient below
                streams.fork(dev, "global")
            conv_dgrad(ds1, pre_n, pre_w, wtn, wtw, dx, dpn, dpw, B, L, KS, dil, BM1, stream)
        if all(dsts[i][1] for i in (0, 1, 2, 3)) and streams.ENABLED:
            # the weight gradient goes to the aux stream: off the critical path, only the optimizer
            # and the DP all-reduce read it (its inputs stay referenced until the join)
            streams.launch(dev, lambda: _wgrad(dpn, dpw, x, KS, dil, 2, B, L, [(dwn, dbn), (dww, dbw)]),
                           keep=[dpn, dpw, x], name="wgrad")
        else:
            _wgrad(dpn, dpw, x, KS, dil, 2, B, L, [(dwn, dbn), (dww, dbw)])
        direct = [p for p, (_, d) in zip(params, dsts) if d]
        if direct:
            notify_grads_ready(direct)
        pgrads = [None if d else g for (g, d) in dsts]
        return (dx, dgb, *pgrads, None, None, None)


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
        _lib.call("pbx_embed_bwd", tok.data_ptr(), d.data_ptr(), dE.data_ptr(), tok.numel(), ctx.V,
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
    """Output buffers of one block's conv weight images and their pack_batch items (v3 form), or
    ``(None, [])`` when the selected conv form packs per call."""
    if CONV_IMPL != "v3":
        return None, []
    KS = wn.shape[2]
    imgs = tuple(torch.empty((KS, CH, CH), dtype=torch.bfloat16, device=wn.device) for _ in range(4))
    return imgs, [(0, wn.detach(), imgs[0], imgs[1], KS, 0), (0, ww.detach(), imgs[2], imgs[3], KS, 0)]


def local_block(x: torch.Tensor, gb: torch.Tensor, blk, packed=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Run the fused local track of ``blk`` (a ``ProteinBERTBlock``)."""
    att = blk.global_attention_layer
    wv = _wv_bf16(att)                                                       # [H*vd, C]
    nc = blk.local_narrow_conv_layer[0]
    wc = blk.local_wide_conv_layer[0]
    return LocalBlockFn.apply(x, gb, nc.weight, nc.bias, wc.weight, wc.bias, blk.local_norm_1.weight,
                              blk.local_norm_1.bias, blk.local_linear_layer[0].weight, blk.local_linear_layer[0].bias,
                              blk.local_norm_2.weight, blk.local_norm_2.bias, wv, blk.wide_conv_dilation, packed)
