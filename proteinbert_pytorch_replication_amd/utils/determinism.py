"""Deterministic mode: bitwise run-to-run reproducible training on the fused HIP path.

By default a few small gradient reductions of the fused path use float atomics whose order depends on
workgroup scheduling, so two runs agree only to rounding:

* ``csrc/ln.hip``    - the [L, C] LayerNorm affine gradients when several workgroups share a position
  pair (L < 2 x #CUs), the broadcast-vector gradient ``dgb`` (one add per 32-position block), the
  embedding gradient;
* ``csrc/glob2.hip`` / ``csrc/glob.hip`` - the global-track LayerNorm / bias / attention-scale column
  sums (one add per 16-row block), the GO input-layer bias gradient.

Everything else is deterministic by construction: the conv weight gradients (``csrc/wgrad.hip``), the
local-MLP weight and bias gradients, the in-tree GEMMs (fixed-order split-K, ``csrc/gemm.hip``), the
heads and their loss partials, the fused Adam and the gradient clipping.

:func:`enable` (or ``PBX_DETERMINISTIC=1`` in the environment) switches those reductions to
fixed-order forms on the same kernels: per-workgroup partial slabs folded by a column-sum launch, and
a single writer per destination for the LayerNorm-affine / ``dgb`` gradients.  The cost is a few
extra small launches per block (``profiles/`` records it).  It also sets
``torch.use_deterministic_algorithms`` for the PyTorch ops around the kernels.  The paper-semantics
kernels and the PyTorch-op fallback for unsupported shapes are not covered by the fixed-order forms.
"""
from __future__ import annotations

import os

import torch

_STATE = {"on": os.environ.get("PBX_DETERMINISTIC", "0") == "1"}


def enable(seed: int = None) -> None:
    """Bitwise-reproducible mode for this process (call before building the model/optimizer)."""
    os.environ.setdefault("CUBLAS_WORKSPACE_CONFIG", ":4096:8")
    torch.use_deterministic_algorithms(True)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    if seed is not None:
        torch.manual_seed(seed)
    _STATE["on"] = True


def disable() -> None:
    _STATE["on"] = False


def enabled() -> bool:
    return _STATE["on"]


def fused_deterministic() -> bool:
    """The fused HIP kernels use their fixed-order reduction forms."""
    return _STATE["on"]


def backend_for(requested: str) -> str:
    """Kernel backend to use (the fused HIP path has a deterministic form: the request stands)."""
    return requested
