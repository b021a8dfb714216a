"""In-tree MFMA GEMMs (``csrc/gemm.hip``) for the library-shaped products of the step.

Every [B, 8943]-wide product of the GO input / output layers, their weight gradients and the
global-track weight gradients ``dW = dU^T X`` run here instead of hipBLASLt:
bf16 operands, fp32 accumulation, 128 x 128 tiles, deterministic split-K (fixed-order slab fold).

``gemm(a, b, out, ta=False, tb=False, accumulate=False)`` computes ``out (+)= op(a) @ op(b)`` where
``op(a) = a`` (``ta=False``, a is [M, K]) or ``a.T`` (``ta=True``, a is [K, M]) and likewise for b
(``tb=True``: b is [N, K]).  Operands are 2-D bf16 tensors with unit inner stride; ``out`` is a 2-D
fp32 tensor with unit inner stride (a view into the flat gradient arena is fine).
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib

_P, _I, _L = ctypes.c_void_p, ctypes.c_int, ctypes.c_long
_lib.register("pbx_gemm", [_P, _L, _I, _P, _L, _I, _P, _L, _I, _I, _I, _I, _I, _I, _P])
_lib.register("pbx_gemm_reduce", [_P, _I, _P, _L, _I, _I, _I, _P])
_lib.register("pbx_go_head_fused", [_P, _L, _P, _L, _P, _P, _L, _P, _P, _P, _L, _P, _P, _I, _I, _I, _P])

BT = 128
BK = 128


def _num_cus(dev) -> int:
    return torch.cuda.get_device_properties(dev).multi_processor_count


def split_count(M: int, N: int, K: int, dev, splitk: Optional[int] = None) -> int:
    """K splits: enough workgroups to cover the CUs when the output has few 128 x 128 tiles (the
    kernel drops empty splits the same way: per = ceil(chunks / s), s' = ceil(chunks / per))."""
    nkc = (K + BK - 1) // BK
    if splitk is None:
        tiles = ((M + BT - 1) // BT) * ((N + BT - 1) // BT)
        splitk = max(1, min(nkc, _num_cus(dev) // max(1, tiles)))
    per = (nkc + splitk - 1) // splitk
    return (nkc + per - 1) // per


def gemm(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, ta: bool = False, tb: bool = False,
         accumulate: bool = False, splitk: Optional[int] = None, k: Optional[int] = None,
         pad_a: bool = False, pad_b: bool = False) -> torch.Tensor:
    """``out[:M, :N] (+)= op(a) @ op(b)``.  ``k``: reduce over the first k entries of the K axis only.
    ``pad_a``/``pad_b``: the operand's memory is zero-padded along its contiguous axis to a multiple
    of 8 elements (lets a [B, 8943] operand stored with an 8960 stride use 16-B loads)."""
    assert a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and out.dtype == torch.float32
    assert a.stride(1) == 1 and b.stride(1) == 1 and out.stride(1) == 1
    M = a.shape[1] if ta else a.shape[0]
    K = a.shape[0] if ta else a.shape[1]
    N = b.shape[0] if tb else b.shape[1]
    Kb = b.shape[1] if tb else b.shape[0]
    if k is not None:
        if k < K and k % 8:
            # the padded path loads whole 8-element chunks: past a ragged k they hold real data
            pad_a = pad_b = False
        K = k
    assert K <= Kb and out.shape[0] >= M and out.shape[1] >= N, (a.shape, b.shape, out.shape, ta, tb)
    dev = a.device
    st = _lib.stream_ptr(dev)
    pad = (1 if pad_a else 0) | (2 if pad_b else 0)
    s = split_count(M, N, K, dev, splitk)
    if s == 1:
        _lib.call("pbx_gemm", a.data_ptr(), a.stride(0), int(ta), b.data_ptr(), b.stride(0), int(tb), out.data_ptr(),
                  out.stride(0), M, N, K, 1, int(accumulate), pad, st)
        return out
    slab = torch.empty((s, M, N), dtype=torch.float32, device=dev)
    _lib.call("pbx_gemm", a.data_ptr(), a.stride(0), int(ta), b.data_ptr(), b.stride(0), int(tb), slab.data_ptr(),
              N, M, N, K, s, 0, pad, st)
    _lib.call("pbx_gemm_reduce", slab.data_ptr(), s, out.data_ptr(), out.stride(0), M, N, int(accumulate), st)
    return out


_lib.register("pbx_gemm_batch", [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p])


def gemm_batch(problems, ta: bool, tb: bool, accumulate: bool = True) -> None:
    """``out_i[:M, :N] (+)= op(a_i) @ op(b_i)`` for up to 4 ``(a, b, out)`` problems of one transpose class
    in ONE launch without split-K (``csrc/gemm.hip`` gemm_batch_kernel)."""
    n = len(problems)
    assert 1 <= n <= 4
    arr = lambda ct, vals: (ct * n)(*vals)  # noqa: E731
    A, B, C, lda, ldb, ldc, M, N, K = ([] for _ in range(9))
    for a, b, out in problems:
        assert a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and out.dtype == torch.float32
        assert a.stride(1) == 1 and b.stride(1) == 1 and out.stride(1) == 1
        m = a.shape[1] if ta else a.shape[0]
        k = a.shape[0] if ta else a.shape[1]
        nn = b.shape[0] if tb else b.shape[1]
        assert (b.shape[1] if tb else b.shape[0]) == k and out.shape[0] >= m and out.shape[1] >= nn
        A.append(a.data_ptr()); B.append(b.data_ptr()); C.append(out.data_ptr())
        lda.append(a.stride(0)); ldb.append(b.stride(0)); ldc.append(out.stride(0))
        M.append(m); N.append(nn); K.append(k)
    P, L64, I32 = ctypes.c_void_p, ctypes.c_long, ctypes.c_int
    _lib.call("pbx_gemm_batch", n, arr(P, A), arr(L64, lda), arr(P, B), arr(L64, ldb), arr(P, C), arr(L64, ldc),
              arr(I32, M), arr(I32, N), arr(I32, K), int(ta), int(tb), int(accumulate),
              _lib.stream_ptr(problems[0][0].device))


def mm(a: torch.Tensor, b: torch.Tensor, ta: bool = False, tb: bool = False, **kw) -> torch.Tensor:
    """New fp32 ``op(a) @ op(b)``."""
    M = a.shape[1] if ta else a.shape[0]
    N = b.shape[0] if tb else b.shape[1]
    out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    return gemm(a, b, out, ta, tb, accumulate=False, **kw)


def go_head_parts(M: int, N: int) -> int:
    """Loss partials written by ``pbx_go_head_fused``: one per 128 x 128 output tile."""
    return ((M + BT - 1) // BT) * ((N + BT - 1) // BT)
