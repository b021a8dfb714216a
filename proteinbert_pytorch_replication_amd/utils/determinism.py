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
``torch.use_deterministic_algorithms`` for the PyTorch ops around the kernels.

The fixed-order forms exist for the reference-semantics kernels with the fused global track
(``glob_fused_ok`` shapes).  The paper-semantics kernels (``csrc/paper_local.hip``) and the general-shape
global track (``csrc/glob.hip``) still reduce with float atomics, so :func:`backend_for` routes those
configurations to the PyTorch path while the mode is on.  ``ProteinBERT.resolved_backend`` applies that
routing with the model's own config on every forward, so it covers ``backend="auto"``, ``bench.py``,
library users and checkpoints loaded under another preset's flags alike.

``PBX_DETERMINISTIC=1`` in the environment is equivalent to calling :func:`enable` at import.
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


def disable() -> None:
    _STATE["on"] = False


def enabled() -> bool:
    return _STATE["on"]


def fused_deterministic() -> bool:
    """The fused HIP kernels use their fixed-order reduction forms."""
    return _STATE["on"]


def fixed_order_supported(model_cfg) -> bool:
    """The fused HIP path has fixed-order forms for this model configuration."""
    if model_cfg is None:
        return True
    get = (lambda k, d=None: model_cfg.get(k, d)) if isinstance(model_cfg, dict) else \
        (lambda k, d=None: getattr(model_cfg, k, d))
    if get("semantics", "reference") == "paper":
        return False
    from ..ops.global_track import glob_fused_ok
    return glob_fused_ok(int(get("global_dim", 512)), int(get("local_dim", 128)))


def backend_for(requested: str, model_cfg=None) -> str:
    """Kernel backend to use.  In deterministic mode a HIP request for a configuration without
    fixed-order kernel forms (paper semantics, unsupported global-track shapes) runs on the PyTorch
    path instead, which ``torch.use_deterministic_algorithms`` makes reproducible."""
    if _STATE["on"] and requested in ("hip", "auto") and not fixed_order_supported(model_cfg):
        if not _STATE.get("warned"):
            import logging
            logging.getLogger(__name__).warning(
                "deterministic mode: no fixed-order HIP kernels for this configuration; using the PyTorch backend")
            _STATE["warned"] = True
        return "torch"
    return requested


if os.environ.get("PBX_DETERMINISTIC", "0") == "1":
    enable()
