"""Global track, input layer and pretraining heads on MI355X (``csrc/glob2.hip``, ``csrc/glob.hip``,
``csrc/gemm.hip``).

Reference: ``ProteinBERT/modules.py:175-199,221-229`` (global MLP + LayerNorm(G)),
``:255-262`` (GO input layer), ``:277-293`` (heads) and ``ProteinBERT/utils.py:293-294`` (loss).

The ``[B, G]`` / ``[B, A]`` products run on the in-tree MFMA GEMM (:mod:`.gemm`: bf16 operands, fp32
accumulation, deterministic split-K); the GO head's GEMM carries the sigmoid / BCE / dlogits epilogue.
Bias, GELU, residual, LayerNorm, the attention scale ``sum(W)/K``, the loss and every elementwise
backward step are fused HIP kernels.  Backward passes are written by hand: each autograd node is a
few launches instead of ~30 eager ops, and parameter gradients accumulate straight into the
flat-arena ``.grad`` views.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Tuple

import torch

from . import _lib, streams
from .gemm import gemm as _gemm, gemm_batch
from .gemm import go_head_parts
from ..parallel import batch_softmax
from ..train.arena import notify_grads_ready
from ..utils.determinism import fused_deterministic

_P, _I, _F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
_lib.register("pbx_row_ln_fwd", [_P, _P, _P, _P, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _I, _I, _F, _P])
_lib.register("pbx_row_ln_bwd", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _I, _I, _P])
_lib.register("pbx_bias_gelu", [_P, _P, _P, _P, _I, _I, _P])
_lib.register("pbx_bias_gelu_bwd", [_P, _P, _P, _P, _P, _I, _I, _P, _P])
_lib.register("pbx_colsum_add", [_P, _I, _I, _P, _P, _P])
_lib.register("pbx_colsum_set", [_P, _I, _I, _P, _P, _P])
_lib.register("pbx_local_head3", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P])
_lib.register("pbx_local_head3_tiles", [_I, _I])
_lib.register("pbx_local_head_fused", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P])
_lib.register("pbx_local_head3_a", [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P])
_lib.register("pbx_local_head3_b", [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P])
_lib.register("pbx_local_head3_c", [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P])
# local head: one launch for B <= 512 (pbx_local_head_fused: 61 vs 108 us for the five-pass form at
# B = L = 512, profiles/r3k_*); larger per-GPU batches take the five-pass form
LHEAD_FUSED = True


def local_head_forward(h: torch.Tensor, wo: torch.Tensor, bo: torch.Tensor, y_l: torch.Tensor, w_l: torch.Tensor,
                       loss_slot: torch.Tensor):
    """Local head + its CE term, reference semantics (softmax over the batch axis; ``csrc/lhead.hip``):
    five coalesced passes over 16-sample x 32-position row tiles.  Writes the mean loss into ``loss_slot``
    and returns (dh [B, L, 128] bf16, dz [B*L, 32] bf16 -- dL/dlogits for the dWo GEMM -- and the
    per-tile bias-gradient partials [tiles, V])."""
    dev = h.device
    st = _s(dev)
    B, L, C = h.shape
    V = wo.shape[0]
    if batch_softmax.active():
        return _local_head_dp(h, wo, bo, y_l, w_l, loss_slot)
    if LHEAD_FUSED and B <= 1024:
        # one launch: a workgroup per 2 positions (B <= 512) or 1 (B <= 1024) x all samples (the batch
        # reductions stay on chip)
        pp = _lib.lib().pbx_local_head_fused_pp(B)
        nt = (L + pp - 1) // pp
        dh = torch.empty_like(h)
        dz = torch.empty((B * L, 32), dtype=BF16, device=dev)
        dbo_part = torch.empty((nt, V), dtype=F32, device=dev)
        lparts = torch.empty(nt, dtype=F32, device=dev)
        _lib.call("pbx_local_head_fused", h.data_ptr(), wo.detach().contiguous().data_ptr(), bo.data_ptr(),
                  y_l.contiguous().data_ptr(), w_l.float().contiguous().data_ptr(), dh.data_ptr(), dz.data_ptr(),
                  dbo_part.data_ptr(), lparts.data_ptr(), B, L, V, st)
        _lib.call("pbx_colsum_set", lparts.data_ptr(), nt, 1, loss_slot.data_ptr(), None, st)
        return dh, dz, dbo_part
    nt = _lib.lib().pbx_local_head3_tiles(B, L)          # the kernel's tile grid (16 samples x 32 positions)
    nch = (B + 15) // 16
    dh = torch.empty_like(h)
    dz = torch.empty((B * L, 32), dtype=BF16, device=dev)
    dbo_part = torch.empty((nt, V), dtype=F32, device=dev)
    lparts = torch.empty(nt, dtype=F32, device=dev)
    Z = torch.empty((B * L, 32), dtype=F32, device=dev)
    part = torch.empty((2, nch, L, 32, 2), dtype=F32, device=dev)
    ms_t = torch.empty((2, L, 32, 2), dtype=F32, device=dev)
    _lib.call("pbx_local_head3", h.data_ptr(), wo.detach().contiguous().data_ptr(), bo.data_ptr(),
              y_l.contiguous().data_ptr(), w_l.float().contiguous().data_ptr(), dh.data_ptr(), dz.data_ptr(),
              dbo_part.data_ptr(), lparts.data_ptr(), Z.data_ptr(), part[0].data_ptr(), part[1].data_ptr(),
              ms_t[0].data_ptr(), ms_t[1].data_ptr(), B, L, V, st)
    _lib.call("pbx_colsum_set", lparts.data_ptr(), nt, 1, loss_slot.data_ptr(), None, st)
    return dh, dz, dbo_part


def _local_head_dp(h, wo, bo, y_l, w_l, loss_slot):
    """The five-pass head with the batch axis of its softmax shared by the data-parallel group
    (``parallel/batch_softmax.py``): stage A leaves the raw (M, S) for the cross-rank merge, stage B's
    T = sum_b G P is summed over ranks before stage C forms dZ = P (G - T)."""
    dev = h.device
    st = _s(dev)
    B, L, C = h.shape
    V = wo.shape[0]
    nt = _lib.lib().pbx_local_head3_tiles(B, L)
    nch = (B + 15) // 16
    dh = torch.empty_like(h)
    dz = torch.empty((B * L, 32), dtype=BF16, device=dev)
    dbo_part = torch.empty((nt, V), dtype=F32, device=dev)
    lparts = torch.empty(nt, dtype=F32, device=dev)
    Z = torch.empty((B * L, 32), dtype=F32, device=dev)
    part = torch.empty((2, nch, L, 32, 2), dtype=F32, device=dev)
    ms_t = torch.empty((2, L, 32, 2), dtype=F32, device=dev)
    wo_c = wo.detach().contiguous()
    y_c = y_l.contiguous()
    w_c = w_l.float().contiguous()
    _lib.call("pbx_local_head3_a", h.data_ptr(), wo_c.data_ptr(), bo.data_ptr(), Z.data_ptr(), part[0].data_ptr(),
              ms_t[0].data_ptr(), 1, B, L, V, st)
    batch_softmax.merge_head_stats(ms_t[0])
    _lib.call("pbx_local_head3_b", Z.data_ptr(), ms_t[0].data_ptr(), y_c.data_ptr(), w_c.data_ptr(),
              part[1].data_ptr(), lparts.data_ptr(), ms_t[1].data_ptr(), B, L, V, st)
    batch_softmax.all_reduce_(ms_t[1], "sum")
    _lib.call("pbx_local_head3_c", Z.data_ptr(), ms_t[0].data_ptr(), ms_t[1].data_ptr(), y_c.data_ptr(),
              w_c.data_ptr(), wo_c.data_ptr(), bo.data_ptr(), dh.data_ptr(), dz.data_ptr(), dbo_part.data_ptr(),
              B, L, V, st)
    _lib.call("pbx_colsum_set", lparts.data_ptr(), nt, 1, loss_slot.data_ptr(), None, st)
    return dh, dz, dbo_part


_lib.register("pbx_glob_bwd", [_P, _I, _I, _I, _I, _P, _P])
_lib.register("pbx_glob3_fwd", [_P, _I, _I, _I, _I, _I, _F, _P])
_lib.register("pbx_pack_glob_frags", [_P, _P, _P, _I, _I, _P])

LN_EPS = 1e-5
BF16 = torch.bfloat16
F32 = torch.float32


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _s(dev) -> int:
    return _lib.stream_ptr(dev)


def bf16_of(p: torch.Tensor) -> torch.Tensor:
    """bf16 copy of a parameter: the optimizer-maintained shadow view when the arena has one."""
    v = getattr(p, "_pbx_bf16", None)
    if v is not None:
        if p._version != p._pbx_bf16_ver:      # written outside the optimizer: refresh the mirror
            # through .data: every mirror is a view of ONE shadow buffer and shares its autograd
            # version counter, so a tracked copy here would invalidate the mirrors of OTHER
            # parameters already saved for backward in this forward pass (their bytes are untouched)
            with torch.no_grad():
                v.data.copy_(p.detach())
            p._pbx_bf16_ver = p._version
        return v
    return p.detach().to(BF16)


def _operand(t: torch.Tensor, inner_axis: int):
    """(base tensor with unit inner stride, transposed?) for a 2-D GEMM operand view: ``t`` itself
    when its last axis is contiguous, else ``t.T`` (a transposed view of a row-major tensor)."""
    if t.stride(1) == 1:
        return t, False
    if t.stride(0) == 1:
        return t.t(), True
    return t.contiguous(), False


def mm32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """bf16 ``a [M, K]`` x bf16 ``b [K, N]`` -> new fp32 [M, N] (in-tree MFMA GEMM; either operand may
    be a transposed view)."""
    out = torch.empty((a.shape[0], b.shape[1]), dtype=F32, device=a.device)
    (a0, ta), (b0, tb) = _operand(a, 1), _operand(b, 1)
    return _gemm(a0, b0, out, ta, tb)


def addmm_into(dst: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> None:
    """dst += a @ b with bf16 operands and fp32 accumulation/output, in place."""
    (a0, ta), (b0, tb) = _operand(a, 1), _operand(b, 1)
    _gemm(a0, b0, dst, ta, tb, accumulate=True)


def addmm_new(c: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """New fp32 ``c + a @ b`` (the incoming ``c`` is left untouched)."""
    out = c.float().clone()
    addmm_into(out, a, b)
    return out


A_ALIGN = 8


def padded_cols(n: int) -> int:
    return (n + A_ALIGN - 1) // A_ALIGN * A_ALIGN


_PAD_CACHE = {}


def bf16_padded(p: torch.Tensor) -> torch.Tensor:
    """bf16 copy of a 2-D parameter ``[R, C]`` with its columns zero-padded to a multiple of 8
    (16-B loads in the MFMA GEMM for odd C such as the 8943 GO annotations); the buffer is cached per
    parameter and refreshed from the bf16 mirror each call.  Returns the ``[R, C]`` view."""
    R, Cc = p.shape
    key = (id(p), p.device)
    buf = _PAD_CACHE.get(key)
    if buf is None or buf.shape != (R, padded_cols(Cc)):
        buf = torch.zeros((R, padded_cols(Cc)), dtype=BF16, device=p.device)
        _PAD_CACHE[key] = buf
    view = buf[:, :Cc]
    view.copy_(bf16_of(p))
    return view


class _Grads:
    """Gradient destinations: arena ``.grad`` views (accumulated in place) or fresh zero tensors."""

    def __init__(self, params):
        self.params = params
        self.dst: List[torch.Tensor] = []
        self.direct: List[bool] = []
        for p in params:
            g = getattr(p, "grad", None) if getattr(p, "_pbx_arena", False) else None
            if g is not None and g.is_contiguous() and g.dtype == F32:
                self.dst.append(g)
                self.direct.append(True)
            elif p is not None and not p.requires_grad:
                # a constant (paper semantics' unit attention weight): the kernels' writes go to scratch
                # nobody reads -- no zero-fill, no gradient returned
                self.dst.append(_scratch_like(p))
                self.direct.append(False)
            else:
                self.dst.append(None if p is None else torch.zeros(p.shape, dtype=F32, device=p.device))
                self.direct.append(False)

    def finish(self):
        direct = [p for p, d in zip(self.params, self.direct) if d and p is not None]
        if direct:
            notify_grads_ready(direct)
        return [None if (d or p is None or not p.requires_grad) else g
                for p, g, d in zip(self.params, self.dst, self.direct)]


_SCRATCH: Dict[Tuple, torch.Tensor] = {}


def _scratch_like(p: torch.Tensor) -> torch.Tensor:
    key = (tuple(p.shape), str(p.device))
    t = _SCRATCH.get(key)
    if t is None:
        t = torch.empty(p.shape, dtype=F32, device=p.device)
        _SCRATCH[key] = t
    return t


_lib.register("pbx_ann_supported", [_I, _I, _I])
_lib.register("pbx_ann_csr", [_P, _I, _I, _P, _P, _P])
_lib.register("pbx_ann_wt", [_P, _P, _I, _I, _P])
_lib.register("pbx_ann_fwd", [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P])
_lib.register("pbx_ann_csc", [_P, _I, _I, _P, _P, _P, _P])
_lib.register("pbx_ann_wgrad", [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P])
# sparse GO input layer (csrc/annot.hip) where pbx_ann_supported; the dense MFMA-GEMM form otherwise
# (tests flip this flag to check both forms)
ANN_SPARSE = True


def ann_sparse_ok(B: int, A: int, G: int) -> bool:
    return ANN_SPARSE and bool(_lib.lib().pbx_ann_supported(B, A, G))


class InputLayerFn(torch.autograd.Function):
    """g0 = GELU(ann W_in^T + b_in) (reference modules.py:255-262,301); ann is the corrupted GO
    multi-hot (values {0, 1, 2} from the corruption, any float accepted).

    Sparse form (default, ``csrc/annot.hip``): the ~0.5 %-dense annotation rows are compacted to
    ordered (column, value) lists and the layer gathers rows of a bf16 ``W^T`` image; the weight
    gradient walks per-column (row, value) lists with ``dU = dG * GELU'(pre)`` kept on chip.  Dense
    form: the in-tree MFMA GEMM on the padded bf16 annotations."""

    @staticmethod
    def forward(ctx, ann, w, b, wgl, bgl):
        dev = ann.device
        st = _s(dev)
        B, A = ann.shape
        G = w.shape[0]
        sparse = ann_sparse_ok(B, A, G)
        if sparse:
            annc = ann.float().contiguous()
            train = any(ctx.needs_input_grad)
            # training: the W^T image and the per-column lists (needed only by the backward) are built on
            # the "ann" aux stream beside the row compaction / the rest of the forward
            aux = train and streams.ENABLED and dev.type == "cuda"
            wt = torch.empty((A, G), dtype=BF16, device=dev)
            wd = w.detach().contiguous()
            if aux:
                with streams.on_aux(dev, "ann", keep=[annc, wd, wt]):
                    _lib.call("pbx_ann_wt", wd.data_ptr(), wt.data_ptr(), G, A, _s(dev))
            else:
                _lib.call("pbx_ann_wt", wd.data_ptr(), wt.data_ptr(), G, A, st)
            cnt = torch.empty(B, dtype=torch.int32, device=dev)
            ent = torch.empty((B * A, 2), dtype=torch.int32, device=dev)
            _lib.call("pbx_ann_csr", annc.data_ptr(), B, A, cnt.data_ptr(), ent.data_ptr(), st)
            if aux:
                streams.wait_for(dev, "ann")
            u = torch.empty((B, G), dtype=F32, device=dev)             # pre-activation, bias included
            g = torch.empty_like(u)
            g_bf = torch.empty((B, G), dtype=BF16, device=dev)
            _lib.call("pbx_ann_fwd", cnt.data_ptr(), ent.data_ptr(), wt.data_ptr(), b.detach().contiguous().data_ptr(),
                      u.data_ptr(), g.data_ptr(), g_bf.data_ptr(), B, A, G, st)
            saved_x = None
            if train:
                ccnt = torch.empty(A, dtype=torch.int32, device=dev)
                cptr = torch.empty(A, dtype=torch.int32, device=dev)
                cent = torch.empty(((A + 63) // 64 * 64 * B, 2), dtype=torch.int32, device=dev)
                if aux:
                    with streams.on_aux(dev, "ann", keep=[annc, ccnt, cptr, cent]):
                        _lib.call("pbx_ann_csc", annc.data_ptr(), B, A, ccnt.data_ptr(), cptr.data_ptr(),
                                  cent.data_ptr(), _s(dev))
                    streams.mark_ready(dev, "ann", [ccnt])
                else:
                    _lib.call("pbx_ann_csc", annc.data_ptr(), B, A, ccnt.data_ptr(), cptr.data_ptr(), cent.data_ptr(),
                              st)
                ctx.csc = (ccnt, cptr, cent, A)
        else:
            # the multi-hot annotations as bf16 ({0, 1, 2} exact) with the columns padded to 8 (16-B loads)
            ann_pad = torch.empty((B, padded_cols(A)), dtype=BF16, device=dev)
            ann_pad[:, A:].zero_()
            ann_bf = ann_pad[:, :A]
            ann_bf.copy_(ann)
            wp = bf16_padded(w)                                                    # [G, A] bf16, padded
            u = torch.empty((B, G), dtype=F32, device=dev)
            _gemm(ann_bf, wp, u, ta=False, tb=True, pad_a=True, pad_b=True)
            g = torch.empty_like(u)
            g_bf = torch.empty((B, G), dtype=BF16, device=dev)
            _lib.call("pbx_bias_gelu", u.data_ptr(), b.data_ptr(), g.data_ptr(), g_bf.data_ptr(), B, G, st)
            saved_x = ann_bf
        # block 0's global->local vector gb = GELU(g Wgl^T + bgl)
        ugl = mm32(g_bf, bf16_of(wgl).t())
        gb = torch.empty_like(ugl)
        _lib.call("pbx_bias_gelu", ugl.data_ptr(), bgl.data_ptr(), gb.data_ptr(), None, B, ugl.shape[1], st)
        ctx.save_for_backward(saved_x, u, g_bf, ugl)
        ctx.params = (w, b, wgl, bgl)
        ctx.sparse = sparse
        ctx.mark_non_differentiable(g_bf)
        ctx.set_materialize_grads(False)     # no zero-filled gradients for unused outputs
        return g, g_bf, gb

    @staticmethod
    def backward(ctx, dg, _dgbf, dgb):
        saved = ctx.saved_tensors
        dev = saved[1].device
        early = dev.type == "cuda" and streams.forked(dev, "ann")
        if early and not all(_Grads(list(ctx.params)).direct):
            streams.cancel_fork(dev, "ann")   # returned gradients are read by autograd on this stream
            early = False
        if early:
            # weight gradients only: the "ann" aux stream (ops/streams.py), forked by the first local
            # block's backward right after dgb was final
            extra = list(ctx.csc[:3]) if getattr(ctx, "csc", None) is not None else []
            with streams.on_aux(dev, "ann", keep=[*saved, dg, dgb, *extra]) as scope:
                out = InputLayerFn._backward(ctx, saved, dg, dgb)
                scope.keep(*[t for t in out if isinstance(t, torch.Tensor)])
            return out
        return InputLayerFn._backward(ctx, saved, dg, dgb)

    @staticmethod
    def _backward(ctx, saved, dg, dgb):
        x, u, g_bf, ugl = saved
        w, b, wgl, bgl = ctx.params
        dev = u.device
        st = _s(dev)
        B, G = u.shape
        gr = _Grads([w, b, wgl, bgl])
        dw, db, dwgl, dbgl = gr.dst
        dg = torch.zeros((B, G), dtype=F32, device=dev) if dg is None else dg.float().contiguous()
        if dgb is not None:
            N = ugl.shape[1]
            dugl = torch.empty((B, N), dtype=BF16, device=dev)
            _lib.call("pbx_bias_gelu_bwd", dgb.float().contiguous().data_ptr(), ugl.data_ptr(), bgl.data_ptr(),
                      dugl.data_ptr(), dbgl.data_ptr(), B, N, _lib.ptr(_det_slab(min(B, BGB_ROWS), N, dev)), st)
            addmm_into(dwgl, dugl.t(), g_bf)
            dg = addmm_new(dg, dugl, bf16_of(wgl))
        if ctx.sparse:
            ccnt, cptr, cent, A = ctx.csc
            streams.wait_ready(ccnt)                # built on the "ann" aux stream in the forward
            streams.queue_join()                    # release the forward's aux-stream keep list
            dut = torch.empty((G, B), dtype=F32, device=dev)
            _lib.call("pbx_ann_wgrad", dg.data_ptr(), u.data_ptr(), ccnt.data_ptr(), cptr.data_ptr(), cent.data_ptr(),
                      dut.data_ptr(), dw.data_ptr(), db.data_ptr(), B, A, G, st)
            del ctx.csc
            return (None, *gr.finish())
        du = torch.empty((B, G), dtype=BF16, device=dev)
        _lib.call("pbx_bias_gelu_bwd", dg.data_ptr(), u.data_ptr(), b.data_ptr(), du.data_ptr(), db.data_ptr(), B, G,
                  _lib.ptr(_det_slab(min(B, BGB_ROWS), G, dev)), st)
        _gemm(du, x, dw, ta=True, tb=False, accumulate=True, pad_b=True)      # dW_in += du^T ann
        return (None, *gr.finish())


# row groups of pbx_bias_gelu_bwd (csrc/glob.hip): a thread walks M / 256 rows (at 32 groups its 32 serial
# row loads made the [1024, 128] input-layer backward an 80 us latency chain in the step's tail)
BGB_ROWS = 256


def _det_slab(rows: int, cols: int, dev) -> Optional[torch.Tensor]:
    """Fixed-order reduction scratch for the deterministic mode (None: in-kernel float atomics)."""
    return torch.empty((rows, cols), dtype=F32, device=dev) if fused_deterministic() else None


def _ptrs(*ts) -> ctypes.Array:
    arr = (ctypes.c_void_p * len(ts))()
    for i, t in enumerate(ts):
        arr[i] = None if t is None else t.data_ptr()
    return arr


# global-track kernels: the column-split forward (csrc/glob3.hip: 3 launches over ceil(B/16) x G/64
# workgroups) and the one-launch backward (csrc/glob2.hip, B/16 workgroups: a column-split backward runs
# beside the conv weight gradient on the aux stream, where its three short launches queued behind the
# weight-gradient workgroups -- 6 + 43 + 45 vs 52 us, profiles/r3h_critpath.txt).  Other shapes take the
# library-GEMM GlobalBlockFn.


def glob_fused_ok(G: int, NGL: int) -> bool:
    """Shapes the fused global-track kernels are compiled for (pbx_glob_supported)."""
    return G in (256, 512) and NGL in (0, 128)


_lib.register("pbx_pack_batch", [_P, _P, _I, _P])
_lib.register("pbx_noop", [_P])


def pack_batch(items) -> None:
    """One launch building every weight image: items are ``(kind, w, out1, out2, n, k)`` with kind 0 =
    conv fragments (``n`` = taps) and kind 1 = Linear fragments (``n`` x ``k``)."""
    if not items:
        return
    for i in range(0, len(items), 40):
        chunk = items[i:i + 40]
        ptrs = (ctypes.c_void_p * (3 * len(chunk)))()
        meta = (ctypes.c_int * (3 * len(chunk)))()
        for j, (kind, w, o1, o2, n, k) in enumerate(chunk):
            ptrs[3 * j], ptrs[3 * j + 1], ptrs[3 * j + 2] = w.data_ptr(), o1.data_ptr(), o2.data_ptr()
            meta[3 * j], meta[3 * j + 1], meta[3 * j + 2] = n, k, kind
        _lib.call("pbx_pack_batch", ptrs, meta, len(chunk), _s(chunk[0][1].device))


def pack_glob(w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """fp32 ``[N, K]`` Linear weight -> bf16 B-fragment images for ``X W^T`` and ``dU W``."""
    N, K = w.shape
    ff = torch.empty((N * K,), dtype=BF16, device=w.device)
    fb = torch.empty_like(ff)
    _lib.call("pbx_pack_glob_frags", w.detach().contiguous().data_ptr(), ff.data_ptr(), fb.data_ptr(), N, K,
              _s(w.device))
    return ff, fb


class FusedGlobalBlockFn(torch.autograd.Function):
    """The global track of one block as ONE kernel forward and ONE kernel backward (``csrc/glob2.hip``;
    the three weight-gradient GEMMs go to the aux stream).  Same math and outputs as
    :class:`GlobalBlockFn`."""

    @staticmethod
    def forward(ctx, g, g_bf, vpart, w1, b1, n1w, n1b, w2, b2, n2w, n2b, wp, wgl, bgl, packed=None):
        """``packed``: the six fragment images (f1, f1T, f2, f2T, fgl, fglT) already built by
        :func:`pack_batch` for this step, else they are built here."""
        dev = g.device
        B, G = g.shape
        TV = vpart.shape[1]
        K = wp.numel()
        NGL = 0 if wgl is None else wgl.shape[0]
        if packed is not None:
            f1, f1T, f2, f2T, fgl, fglT = packed
        else:
            f1, f1T = pack_glob(w1)
            f2, f2T = pack_glob(w2)
            fgl, fglT = pack_glob(wgl) if NGL else (None, None)
        e = lambda *shape, dt=F32: torch.empty(shape, dtype=dt, device=dev)  # noqa: E731
        pre1, xh1, vsum, pre2, xh2, g2 = e(B, G), e(B, G), e(B, G), e(B, G), e(B, G), e(B, G)
        r1, r2 = e(B), e(B)
        g1_bf, g2_bf = e(B, G, dt=BF16), e(B, G, dt=BF16)
        pregl, gb = (e(B, NGL), e(B, NGL)) if NGL else (None, torch.zeros((B, 0), dtype=F32, device=dev))
        vp, TVk = vpart.contiguous(), TV
        if TV > 16:
            # long sequences: the attention-pool tile partials are summed by the whole chip first (the
            # fused kernel has only B / 16 workgroups; at L = 4096 each would stream 64 tile rows)
            vp, TVk = vp.sum(dim=1, keepdim=True), 1
        gc, gbc = g.contiguous(), g_bf.contiguous()

        NCT = G // 64
        z1, z2 = e(B, G), e(B, G)
        part1, part2 = e(B, NCT, 2), e(B, NCT, 2)
        _lib.call("pbx_glob3_fwd", _ptrs(gc, gbc, vp, wp, f1, b1, n1w, n1b, f2, b2, n2w, n2b,
                                         fgl, bgl, pre1, xh1, r1, vsum, g1_bf, pre2, xh2, r2, g2, g2_bf, pregl,
                                         gb if NGL else None, z1, z2, part1, part2),
                  B, G, NGL, TVk, K, LN_EPS, _s(dev))
        ctx.save_for_backward(g_bf, pre1, xh1, r1, vsum, g1_bf, pre2, xh2, r2, g2_bf, pregl, f1T, f2T, fglT)
        ctx.params = (w1, b1, n1w, n1b, w2, b2, n2w, n2b, wp, wgl, bgl)
        ctx.meta = (TV, NGL)
        ctx.mark_non_differentiable(g2_bf)
        ctx.set_materialize_grads(False)
        return g2, g2_bf, gb

    @staticmethod
    def backward(ctx, dg2, _dg2bf, dgb):
        return FusedGlobalBlockFn._backward(ctx, ctx.saved_tensors, dg2, dgb)

    @staticmethod
    def _backward(ctx, saved, dg2, dgb):
        g_bf, pre1, xh1, r1, vsum, g1_bf, pre2, xh2, r2, g2_bf, pregl, f1T, f2T, fglT = saved
        w1, b1, n1w, n1b, w2, b2, n2w, n2b, wp, wgl, bgl = ctx.params
        TV, NGL = ctx.meta
        dev = pre1.device
        B, G = pre1.shape
        gr = _Grads([w1, b1, n1w, n1b, w2, b2, n2w, n2b, wp, wgl, bgl])
        dw1, db1, dn1w, dn1b, dw2, db2, dn2w, dn2b, dwp, dwgl, dbgl = gr.dst
        dg2 = torch.zeros((B, G), dtype=F32, device=dev) if dg2 is None else dg2.float().contiguous()
        if NGL:
            dgb = torch.zeros((B, NGL), dtype=F32, device=dev) if dgb is None else dgb.float().contiguous()
        else:
            dgb = None
        dg = torch.empty((B, G), dtype=F32, device=dev)
        dvs = torch.empty((B, G), dtype=F32, device=dev)
        du1 = torch.empty((B, G), dtype=BF16, device=dev)
        du2 = torch.empty((B, G), dtype=BF16, device=dev)
        dugl = torch.empty((B, NGL), dtype=BF16, device=dev) if NGL else None
        _lib.call("pbx_glob_bwd", _ptrs(dg2, dgb, pregl, fglT, xh2, r2, n2w, pre2, f2T, xh1, r1, n1w, pre1, vsum,
                                        wp, f1T, dg, dvs, du1, du2, dugl, db1, dn1w, dn1b, db2, dn2w, dn2b,
                                        dbgl if NGL else None, dwp),
                  B, G, NGL, wp.numel(), _lib.ptr(_det_slab((B + 15) // 16, 6 * G + NGL + wp.numel(), dev)),
                  _s(dev))

        def weight_grads():
            # dW = dU^T X for W1, W2 and the next block's global->local weight: one batched launch,
            # K = B rows, accumulated straight into the gradient destinations (no split-K slabs)
            probs = [(du1, g_bf, dw1), (du2, g1_bf, dw2)] + ([(dugl, g2_bf, dwgl)] if NGL else [])
            if all(d.is_contiguous() and d.dtype == F32 for _, _, d in probs):
                gemm_batch(probs, ta=True, tb=False, accumulate=True)
            else:
                for a, b, d in probs:
                    addmm_into(d, a.t(), b)

        direct = all(gr.direct[i] for i in (0, 4)) and (not NGL or gr.direct[9])
        if direct and streams.ENABLED and dev.type == "cuda":
            # dW = dU^T X (K = B rows) is off the critical path: the aux (weight-gradient) stream
            streams.launch(dev, weight_grads, keep=[du1, du2, dugl, g_bf, g1_bf, g2_bf], name="wgrad")
        else:
            weight_grads()
        dvpart = dvs.unsqueeze(1).expand(B, TV, G)
        return (dg, None, dvpart, *gr.finish(), None, None)


class GlobalBlockFn(torch.autograd.Function):
    """Global track of one block (reference modules.py:175-199,219-229, reference semantics):

        g1 = LN1(g + GELU(g W1^T + b1) + (sum W_att / K) * sum_t vpart)
        g2 = LN2(g1 + GELU(g1 W2^T + b2))
        gb_next = GELU(g2 Wgl_next^T + bgl_next)      (the next block's global->local vector)
    """

    @staticmethod
    def forward(ctx, g, g_bf, vpart, w1, b1, n1w, n1b, w2, b2, n2w, n2b, wp, wgl, bgl):
        dev = g.device
        B, G = g.shape
        TV = vpart.shape[1]
        K = wp.numel()
        st = _s(dev)
        u1 = mm32(g_bf, bf16_of(w1).t())
        g1 = torch.empty_like(g)
        g1_bf = torch.empty((B, G), dtype=BF16, device=dev)
        xh1 = torch.empty_like(g)
        r1 = torch.empty(B, dtype=F32, device=dev)
        vsum = torch.empty_like(g)
        _lib.call("pbx_row_ln_fwd", u1.data_ptr(), b1.data_ptr(), g.data_ptr(), vpart.data_ptr(), TV, wp.data_ptr(),
                  K, n1w.data_ptr(), n1b.data_ptr(), g1.data_ptr(), g1_bf.data_ptr(), xh1.data_ptr(), r1.data_ptr(),
                  vsum.data_ptr(), B, G, LN_EPS, st)
        u2 = mm32(g1_bf, bf16_of(w2).t())
        g2 = torch.empty_like(g)
        g2_bf = torch.empty((B, G), dtype=BF16, device=dev)
        xh2 = torch.empty_like(g)
        r2 = torch.empty(B, dtype=F32, device=dev)
        _lib.call("pbx_row_ln_fwd", u2.data_ptr(), b2.data_ptr(), g1.data_ptr(), None, 0, None, 0, n2w.data_ptr(),
                  n2b.data_ptr(), g2.data_ptr(), g2_bf.data_ptr(), xh2.data_ptr(), r2.data_ptr(), None, B, G, LN_EPS,
                  st)
        if wgl is not None:
            ugl = mm32(g2_bf, bf16_of(wgl).t())
            N = ugl.shape[1]
            gb = torch.empty_like(ugl)
            _lib.call("pbx_bias_gelu", ugl.data_ptr(), bgl.data_ptr(), gb.data_ptr(), None, B, N, st)
        else:
            ugl = None
            gb = torch.zeros((B, 0), dtype=F32, device=dev)
        ctx.save_for_backward(g_bf, u1, xh1, r1, vsum, g1_bf, u2, xh2, r2, g2_bf, ugl)
        ctx.params = (w1, b1, n1w, n1b, w2, b2, n2w, n2b, wp, wgl, bgl)
        ctx.TV = TV
        ctx.mark_non_differentiable(g2_bf)
        ctx.set_materialize_grads(False)
        return g2, g2_bf, gb

    @staticmethod
    def backward(ctx, dg2, _dg2bf, dgb):
        return GlobalBlockFn._backward(ctx, ctx.saved_tensors, dg2, dgb)

    @staticmethod
    def _backward(ctx, saved, dg2, dgb):
        g_bf, u1, xh1, r1, vsum, g1_bf, u2, xh2, r2, g2_bf, ugl = saved
        w1, b1, n1w, n1b, w2, b2, n2w, n2b, wp, wgl, bgl = ctx.params
        dev = u1.device
        st = _s(dev)
        B, G = u1.shape
        gr = _Grads([w1, b1, n1w, n1b, w2, b2, n2w, n2b, wp, wgl, bgl])
        dw1, db1, dn1w, dn1b, dw2, db2, dn2w, dn2b, dwp, dwgl, dbgl = gr.dst
        dg2 = torch.zeros((B, G), dtype=F32, device=dev) if dg2 is None else dg2.float().contiguous()
        if wgl is not None and dgb is not None and dgb.numel() > 0:
            N = ugl.shape[1]
            dugl = torch.empty((B, N), dtype=BF16, device=dev)
            _lib.call("pbx_bias_gelu_bwd", dgb.float().contiguous().data_ptr(), ugl.data_ptr(), bgl.data_ptr(),
                      dugl.data_ptr(), dbgl.data_ptr(), B, N, _lib.ptr(_det_slab(min(B, BGB_ROWS), N, dev)), st)
            addmm_into(dwgl, dugl.t(), g2_bf)
            dg2 = addmm_new(dg2, dugl, bf16_of(wgl))                   # new buffer (incoming grad untouched)
        # LN2 + MLP2
        du2 = torch.empty((B, G), dtype=BF16, device=dev)
        dg1 = torch.empty((B, G), dtype=F32, device=dev)
        _lib.call("pbx_row_ln_bwd", dg2.data_ptr(), xh2.data_ptr(), r2.data_ptr(), n2w.data_ptr(), u2.data_ptr(),
                  b2.data_ptr(), dn2w.data_ptr(), dn2b.data_ptr(), db2.data_ptr(), du2.data_ptr(), dg1.data_ptr(),
                  None, None, 0, None, None, B, G, st)
        addmm_into(dw2, du2.t(), g1_bf)
        addmm_into(dg1, du2, bf16_of(w2))
        # LN1 + MLP1 + attention scale
        du1 = torch.empty((B, G), dtype=BF16, device=dev)
        dg = torch.empty((B, G), dtype=F32, device=dev)
        dvs = torch.empty((B, G), dtype=F32, device=dev)
        _lib.call("pbx_row_ln_bwd", dg1.data_ptr(), xh1.data_ptr(), r1.data_ptr(), n1w.data_ptr(), u1.data_ptr(),
                  b1.data_ptr(), dn1w.data_ptr(), dn1b.data_ptr(), db1.data_ptr(), du1.data_ptr(), dg.data_ptr(),
                  vsum.data_ptr(), wp.data_ptr(), wp.numel(), dwp.data_ptr(), dvs.data_ptr(), B, G, st)
        addmm_into(dw1, du1.t(), g_bf)
        addmm_into(dg, du1, bf16_of(w1))
        dvpart = dvs.unsqueeze(1).expand(B, ctx.TV, G)
        return (dg, None, dvpart, *gr.finish())


# the GO head's forward runs on the "head" aux stream beside the local head (when aux streams are on)


class HeadsLossFn(torch.autograd.Function):
    """Both pretraining heads + the reference loss (``utils.py:293-294``), reference semantics.

    The loss is terminal, so both heads compute their input gradients in the forward pass: the
    local-head kernel writes dh, and the GO head is ONE MFMA GEMM launch whose epilogue evaluates
    sigmoid / BCE / dlogits and the bias-gradient partials (``csrc/gemm.hip`` EPI_GO: the [B, 8943]
    logits never reach memory).  The backward is two in-tree GEMMs (dg2 = dz Wa, dWa += dz^T g2).
    """

    @staticmethod
    def forward(ctx, h, g2, g2_bf, wo, bo, wa, ba, y_l, y_g, w_l, w_g):
        dev = h.device
        st = _s(dev)
        B, L, C = h.shape
        V = wo.shape[0]
        A = wa.shape[0]
        loss = torch.empty(2, dtype=F32, device=dev)        # each head writes its slot (pbx_colsum_set)
        if streams.ENABLED and dev.type == "cuda":
            # the GO head (GEMM + VALU-heavy BCE epilogue) on its own stream beside the memory-bound
            # local head; the loss sum waits for both
            res = []

            def go():
                res.append(go_head_forward(g2_bf, wa, ba, y_g, w_g, loss[1:]))
                return list(res[0])

            streams.launch(dev, go, keep=[g2_bf, wa, ba, y_g, w_g, loss], name="head")
            dh, dzl, dbo_part = local_head_forward(h, wo, bo, y_l, w_l, loss[0:1])
            streams.wait_for(dev, "head")
            dz, dba, gx = res[0]
        else:
            dh, dzl, dbo_part = local_head_forward(h, wo, bo, y_l, w_l, loss[0:1])
            dz, dba, gx = go_head_forward(g2_bf, wa, ba, y_g, w_g, loss[1:])
        ctx.save_for_backward(dh, dzl, dbo_part, h, dz, dba, gx)
        ctx.params = (wo, bo, wa, ba)
        ctx.V = V
        total = loss_total(loss)
        ctx.mark_non_differentiable(loss)
        ctx.set_materialize_grads(False)
        return total, loss

    @staticmethod
    def backward(ctx, dtotal, _dparts):
        dh, dzl, dbo_part, h, dz, dba, g2_bf = ctx.saved_tensors
        wo, bo, wa, ba = ctx.params
        gr = _Grads([wo, bo, wa, ba])
        dwo, dbo_dst, dwa, dba_dst = gr.dst
        st = _s(dh.device)
        if dtotal is None:
            return (None,) * 11
        if _UNIT_LOSS_GRAD[0]:
            # loss.backward() from the training step: d(loss) == 1 exactly, skip the rescale passes
            dh_s, scale = dh, None
        else:
            scale = dtotal.reshape(1).to(F32).contiguous()
            dh_s = (dh.float() * scale.reshape(())).to(dh.dtype)
        # weight gradients (dWo = dzl^T h with K = B*L, dbo, dWa = dz^T g2, dba) feed only the optimizer
        # and the DP all-reduce: on the aux weight-gradient stream, beside the critical-path dg2 GEMM and
        # the last block's backward
        V = wo.shape[0]
        hr = h.reshape(-1, h.shape[-1])

        def weight_grads():
            if scale is None:
                _gemm(dzl[:, :V], hr, dwo, ta=True, tb=False, accumulate=True, pad_a=True)
            else:
                dwo.add_(_gemm(dzl[:, :V], hr, torch.empty_like(dwo), ta=True, tb=False, pad_a=True) * scale)
            _lib.call("pbx_colsum_add", dbo_part.data_ptr(), dbo_part.shape[0], V, dbo_dst.data_ptr(),
                      _lib.ptr(scale), _s(dh.device))
            go_head_weight_grads(dz_s, dba, g2_bf, dwa, dba_dst, scale)

        dz_s = go_head_scaled_dz(dz, scale)
        if all(gr.direct) and streams.ENABLED and dh.device.type == "cuda":
            streams.launch(dh.device, weight_grads, keep=[dzl, h, dbo_part, dz_s, dba, g2_bf], name="wgrad")
        else:
            weight_grads()
        dg2 = go_head_input_grad(dz_s, g2_bf, wa)

        return (dh_s, dg2, None, *gr.finish(), None, None, None, None)


def go_head_forward(g2_bf: torch.Tensor, wa: torch.Tensor, ba: torch.Tensor, y_g: torch.Tensor,
                    w_g: torch.Tensor, loss_slot: torch.Tensor):
    """GO head + its BCE term (reference ``modules.py:286-293``, ``utils.py:294``) as ONE launch:
    z = g2 Wa^T + ba, sigmoid, BCE with the log clamp, weight, dz = dL/dz (bf16) and the bias-gradient
    partials (``pbx_go_head_fused``); the mean loss is written into ``loss_slot`` (device scalar).
    Returns (dz [B, A] view of a column-padded buffer, bias-gradient partials [ceil(B/128), A], g2)."""
    dev = g2_bf.device
    st = _s(dev)
    B, A = g2_bf.shape[0], wa.shape[0]
    dz_pad = torch.empty((B, padded_cols(A)), dtype=BF16, device=dev)     # pad columns zeroed by the kernel
    dz = dz_pad[:, :A]
    dba = torch.empty(((B + 127) // 128, A), dtype=F32, device=dev)
    lparts = torch.empty(go_head_parts(B, A), dtype=F32, device=dev)
    y = y_g.float().contiguous()
    # per-row weights (the reference's any(annotation) broadcast) are read without expanding them
    if w_g.dim() == 2 and w_g.stride(1) == 0:
        wrow, wfull = w_g[:, 0].float().contiguous(), None
    else:
        wrow, wfull = None, w_g.float().expand(B, A).contiguous()
    gx = g2_bf.contiguous()
    wab = bf16_of(wa)
    _lib.call("pbx_go_head_fused", gx.data_ptr(), gx.stride(0), wab.data_ptr(), wab.stride(0), ba.data_ptr(),
              y.data_ptr(), A, _lib.ptr(wrow), _lib.ptr(wfull), dz.data_ptr(), dz_pad.stride(0), dba.data_ptr(),
              lparts.data_ptr(), B, A, gx.shape[1], st)
    _lib.call("pbx_colsum_set", lparts.data_ptr(), lparts.numel(), 1, loss_slot.data_ptr(), None, st)
    return dz, dba, gx


def go_head_scaled_dz(dz, scale=None):
    """dz times the incoming loss gradient (device [1]) when it is not exactly 1 (column-padded copy)."""
    if scale is None:
        return dz
    B, A = dz.shape
    dz_s = torch.zeros((B, padded_cols(A)), dtype=BF16, device=dz.device)[:, :A]
    dz_s.copy_(dz.float() * scale.reshape(()))
    return dz_s


def go_head_input_grad(dz_s, g2_bf, wa) -> torch.Tensor:
    """dg2 = dz Wa (K = A: split-K)."""
    dg2 = torch.empty((dz_s.shape[0], g2_bf.shape[1]), dtype=F32, device=dz_s.device)
    _gemm(dz_s, bf16_of(wa), dg2, ta=False, tb=False, pad_a=True)
    return dg2


def go_head_weight_grads(dz_s, dba, g2_bf, dwa_dst, dba_dst, scale=None) -> None:
    """dWa += dz^T g2, dba += s sum_rows(dz) (from the per-row-tile partials)."""
    A = dz_s.shape[1]
    _lib.call("pbx_colsum_add", dba.data_ptr(), dba.shape[0], A, dba_dst.data_ptr(), _lib.ptr(scale), _s(dz_s.device))
    _gemm(dz_s, g2_bf, dwa_dst, ta=True, tb=False, accumulate=True, pad_a=True)


def go_head_backward(dz, dba, g2_bf, wa, dwa_dst, dba_dst, scale=None) -> torch.Tensor:
    """dg2 = s dz Wa (K = A: split-K), dWa += s dz^T g2, dba += s sum_rows(dz); ``scale`` (device
    [1] or None) = the incoming gradient of the loss."""
    dz_s = go_head_scaled_dz(dz, scale)
    go_head_weight_grads(dz_s, dba, g2_bf, dwa_dst, dba_dst, scale)
    return go_head_input_grad(dz_s, g2_bf, wa)


_UNIT_LOSS_GRAD = [False]


def loss_total(loss: torch.Tensor) -> torch.Tensor:
    """loss[0] + loss[1] as a 0-d device tensor (one in-tree launch: the fixed-order column sum)."""
    if loss.is_cuda:
        total = torch.empty((), dtype=F32, device=loss.device)
        _lib.call("pbx_colsum_set", loss.data_ptr(), loss.numel(), 1, total.data_ptr(), None, _s(loss.device))
        return total
    return loss.sum()


_ONES = {}


def unit_seed(t: torch.Tensor) -> torch.Tensor:
    """A cached device 1.0 of ``t``'s shape / dtype: ``torch.autograd.backward(loss, unit_seed(loss))`` starts
    the backward without the fill kernel autograd's implicit seed launches every step."""
    key = (t.device, t.dtype, tuple(t.shape))
    v = _ONES.get(key)
    if v is None:
        v = _ONES[key] = torch.ones(t.shape, dtype=t.dtype, device=t.device)
    return v


class unit_loss_grad:
    """Context for ``loss.backward()`` with the implicit gradient 1.0 (the training step): lets the
    fused loss skip scaling its precomputed gradients by d(loss)."""

    def __enter__(self):
        self._prev = _UNIT_LOSS_GRAD[0]
        _UNIT_LOSS_GRAD[0] = True
        return self

    def __exit__(self, *exc):
        _UNIT_LOSS_GRAD[0] = self._prev
        return False
