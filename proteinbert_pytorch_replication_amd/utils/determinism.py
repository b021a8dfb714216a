"""Deterministic mode: bitwise run-to-run reproducible training.

The fused HIP path reduces several gradients with float atomics whose order depends on workgroup
scheduling, so two runs agree only to rounding (bounded, tested in ``tests/test_determinism.py``):

* ``csrc/ln.hip``   - local-MLP ``dWl``/``dbl`` (one flush per position-pair workgroup), the [L, C]
  LayerNorm affine gradients when more than one workgroup shares a position pair (L < 2 x #CUs),
  the broadcast-vector gradient ``dgb`` (one add per 32-position block), the embedding gradient;
* ``csrc/glob.hip`` / ``csrc/glob2.hip`` - global-track LayerNorm / bias gradients (one add per
  16-row block), the local-head column sum of G*P (LDS atomics across waves), the GO-head bias
  gradient, the loss scalars;
* library GEMMs that select split-K algorithms.

The conv weight gradients (the largest reduction, ``csrc/wgrad.hip``) use fixed-order slab
reductions and are deterministic.  :func:`enable` switches a run to the PyTorch path with
``torch.use_deterministic_algorithms`` (same model, same semantics, eager speed); the fused Adam,
gradient clipping (two-phase sum of squares) and data generation kernels are deterministic.
"""
from __future__ import annotations

import os

import torch

_STATE = {"on": False}


def enable(seed: int = None) -> None:
    """Bitwise-reproducible mode for this process (call before building the model/optimizer)."""
    os.environ.setdefault("CUBLAS_WORKSPACE_CONFIG", ":4096:8")
    torch.use_deterministic_algorithms(True)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    if seed is not None:
        torch.manual_seed(seed)
    _STATE["on"] = True


def enabled() -> bool:
    return _STATE["on"]


def backend_for(requested: str) -> str:
    """Kernel backend to use: the PyTorch path whenever deterministic mode is on."""
    return "torch" if _STATE["on"] else requested
