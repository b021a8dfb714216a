"""Paper-semantics global attention as a differentiable composition around the split-L HIP core.

The published ProteinBERT attention (one query per head from the global track, softmax over the
sequence axis, pad-masked) that the reference's ``GlobalAttentionHead`` (``ProteinBERT/modules.py:49-60``)
was written to compute; the reference's own softmax axis makes it a mean pool instead,
which is what ``semantics="reference"`` reproduces.

Split of the work:

* ``q = tanh(g Wq) / sqrt(K)`` and ``pre = h [Wk | Wv]`` are autograd matmuls (this function serves the
  eager model's ``use_kernel`` path, :meth:`..models.proteinbert.GlobalAttention.forward_paper`);
* tanh / GELU / scores / masked softmax / P.V, and the whole backward of that chain, are the
  split-L HIP kernels (:func:`paper_attention_core`).

The training executor does not use this composition: :class:`.paper_track.PaperBlockFn` runs the
K/V projections inside the fused attention kernels (``csrc/paper_fused.hip``) and every remaining GEMM
on the in-tree MFMA GEMM (``csrc/gemm.hip``).

The torch oracle is :meth:`...models.proteinbert.GlobalAttention.forward_paper` with ``use_kernel=False``.
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional

import torch

from . import _lib

_P, _I = ctypes.c_void_p, ctypes.c_int
_lib.register("pbx_paper_attn_fwd", [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P])
_lib.register("pbx_paper_attn_bwd", [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P])

KEY_DIM = 64
VALUE_DIM = 128
# False: every call takes the torch oracle (parity tests flip it)
ENABLED = True


def kernel_supported(h: torch.Tensor, key_dim: int, value_dim: int) -> bool:
    """Shapes/dtypes the HIP core is written for (the paper config: K=64, VD=128, bf16 on a GPU)."""
    return ENABLED and h.is_cuda and h.dtype == torch.bfloat16 and key_dim == KEY_DIM and value_dim == VALUE_DIM


def _nsplit(B: int, H: int, L: int) -> int:
    # >= ~2048 workgroups over the 256 CUs, chunks of >= 64 positions
    want = max(1, -(-4096 // (B * H)))
    ns = max(1, min(want, -(-L // 64)))
    chunk = -(-L // ns)
    return -(-L // chunk)                     # every chunk non-empty


class _PaperAttnCore(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pre: torch.Tensor, qs: torch.Tensor, mask: Optional[torch.Tensor], H: int):
        B, L, N = pre.shape
        assert N == H * (KEY_DIM + VALUE_DIM) and pre.dtype == torch.bfloat16 and pre.is_contiguous()
        assert qs.shape == (B, H, KEY_DIM) and qs.dtype == torch.float32 and qs.is_contiguous()
        if mask is not None:
            assert mask.shape == (B, L) and mask.dtype == torch.bool and mask.is_contiguous()
        ns = _nsplit(B, H, L)
        part = torch.empty(B * H, ns, 2 + VALUE_DIM, device=pre.device, dtype=torch.float32)
        o = torch.empty(B, H * VALUE_DIM, device=pre.device, dtype=torch.float32)
        lse = torch.empty(B * H, device=pre.device, dtype=torch.float32)
        _lib.call("pbx_paper_attn_fwd", pre.data_ptr(), qs.data_ptr(), _lib.ptr(mask), part.data_ptr(),
                  o.data_ptr(), lse.data_ptr(), B, L, H, KEY_DIM, VALUE_DIM, ns, _lib.stream_ptr(pre.device))
        ctx.save_for_backward(pre, qs, mask, o, lse)
        ctx.H, ctx.ns = H, ns
        return o

    @staticmethod
    def backward(ctx, dO: torch.Tensor):
        pre, qs, mask, o, lse = ctx.saved_tensors
        B, L, _ = pre.shape
        H, ns = ctx.H, ctx.ns
        dO = dO.float().contiguous()
        dpre = torch.empty_like(pre)
        dq_part = torch.empty(B * H, ns, KEY_DIM, device=pre.device, dtype=torch.float32)
        _lib.call("pbx_paper_attn_bwd", pre.data_ptr(), qs.data_ptr(), _lib.ptr(mask), lse.data_ptr(),
                  o.data_ptr(), dO.data_ptr(), dpre.data_ptr(), dq_part.data_ptr(), B, L, H, KEY_DIM,
                  VALUE_DIM, ns, _lib.stream_ptr(pre.device))
        dqs = dq_part.sum(dim=1).view(B, H, KEY_DIM)
        return dpre, dqs, None, None


def paper_attention_core(pre: torch.Tensor, qs: torch.Tensor, mask: Optional[torch.Tensor], H: int) -> torch.Tensor:
    """``o[b, h*VD:(h+1)*VD] = sum_l softmax_l(qs[b,h] . tanh(pre_k[b,l,h])) GELU(pre_v[b,l,h])``."""
    return _PaperAttnCore.apply(pre, qs, mask, H)


def paper_attention(h: torch.Tensor, g: torch.Tensor, Wq: torch.Tensor, Wk: torch.Tensor, Wv: torch.Tensor,
                    mask: Optional[torch.Tensor]) -> torch.Tensor:
    """Full paper attention ``[B, L, C] x [B, G] -> [B, H*VD]`` (fp32) with the HIP core."""
    H, C, K = Wk.shape
    VD = Wv.shape[2]
    B, L, _ = h.shape
    q = torch.tanh(torch.einsum("bg,hgk->bhk", g.float(), Wq.float()))
    qs = (q * (1.0 / math.sqrt(K))).contiguous()
    wcat = torch.cat([Wk.permute(1, 0, 2).reshape(C, H * K), Wv.permute(1, 0, 2).reshape(C, H * VD)], dim=1)
    pre = torch.matmul(h.reshape(B * L, C), wcat.to(h.dtype)).view(B, L, H * (K + VD))
    return paper_attention_core(pre, qs, None if mask is None else mask.contiguous(), H)
