"""Fused on-device synthetic batch generation + corruption (HIP ``data.hip``).

Same distributions as :func:`..data.synthetic.corrupt_batch_torch` (the
oracle) and the reference per-sample transforms
(``ProteinBERT/data_processing.py:86-180``).  ``W["global"]`` is returned as a
zero-copy ``[B, A]`` broadcast of a per-sample ``[B]`` weight.
"""
from __future__ import annotations

import ctypes
from typing import Tuple

import torch

from . import _lib
from ..data.vocab import VOCAB_SIZE

_P, _I, _F, _U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_uint64
_lib.register("pbx_synth_batch", [_P, _P, _I, _I, _I, _I, _I, _F, _I, _U64, _U64, _P, _P])
_lib.register("pbx_corrupt_batch", [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _F, _F, _F, _F, _U64, _U64, _P, _P])


def _check(t: torch.Tensor, dtype, name: str):
    if not t.is_cuda or t.dtype != dtype or not t.is_contiguous():
        raise ValueError(f"{name}: expected contiguous {dtype} CUDA tensor, got {t.dtype} {t.device}")


def synth_batch(B: int, L: int, A: int, min_len: int, max_len: int, density: float, seed: int, step: int,
                device, step_dev: torch.Tensor = None) -> Tuple[torch.Tensor, torch.Tensor]:
    tokens = torch.empty((B, L), dtype=torch.long, device=device)
    ann = torch.empty((B, A), dtype=torch.float32, device=device)
    if max_len < min_len:
        raise ValueError("max_len < min_len")
    _lib.call("pbx_synth_batch", tokens.data_ptr(), ann.data_ptr(), B, L, A, min_len, max_len, float(density),
              VOCAB_SIZE, seed & (2**64 - 1), step, _lib.ptr(step_dev), _lib.stream_ptr(tokens.device))
    return tokens, ann


def corrupt_batch(tokens: torch.Tensor, ann: torch.Tensor, params, seed: int, step: int,
                  step_dev: torch.Tensor = None):
    _check(tokens, torch.long, "tokens")
    _check(ann, torch.float32, "ann")
    B, L = tokens.shape
    if ann.shape[0] != B:
        raise ValueError("batch mismatch")
    A = ann.shape[1]
    x_local = torch.empty_like(tokens)
    x_global = torch.empty_like(ann)
    w_local = torch.empty((B, L), dtype=torch.float32, device=tokens.device)
    w_sample = torch.empty((B,), dtype=torch.float32, device=tokens.device)
    _lib.call("pbx_corrupt_batch", tokens.data_ptr(), ann.data_ptr(), x_local.data_ptr(), x_global.data_ptr(),
              w_local.data_ptr(), w_sample.data_ptr(), B, L, A, VOCAB_SIZE, float(params.token_p),
              float(params.positive_p), float(params.negative_p), float(params.blank_p),
              seed & (2**64 - 1), step, _lib.ptr(step_dev), _lib.stream_ptr(tokens.device))
    return ({"local": x_local, "global": x_global},
            {"local": tokens, "global": ann},
            {"local": w_local, "global": w_sample.unsqueeze(1).expand(B, A)})


_lib.register("pbx_unpack_batch", [_P, _P, _P, _P, _I, _I, _I, _I, _P])


def unpack_batch(tok_u8: torch.Tensor, bits: torch.Tensor, A: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Expand a compact loader batch on the device: u8 tokens -> int64, annotation bits -> f32."""
    _check(tok_u8, torch.uint8, "tok_u8")
    _check(bits, torch.uint8, "bits")
    B, L = tok_u8.shape
    nbytes = bits.shape[1]
    if bits.shape[0] != B or nbytes * 8 < A:
        raise ValueError("bits shape does not cover the annotation count")
    tokens = torch.empty((B, L), dtype=torch.long, device=tok_u8.device)
    ann = torch.empty((B, A), dtype=torch.float32, device=tok_u8.device)
    _lib.call("pbx_unpack_batch", tok_u8.data_ptr(), bits.data_ptr(), tokens.data_ptr(), ann.data_ptr(), B, L, A,
              nbytes, _lib.stream_ptr(tok_u8.device))
    return tokens, ann
