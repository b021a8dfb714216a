"""Flat parameter / gradient arena.

All trainable parameters are re-pointed into ONE contiguous fp32 buffer and
their ``.grad`` tensors into a second one.  This is what makes the MI355X
step cheap outside the model:

* the optimizer is a single fused launch over the arena (``ops.optim``),
* DP gradient buckets are contiguous slices of the grad arena, all-reduced
  in place by RCCL without copies (``parallel.ddp``),
* grad zeroing is one memset, grad-norm clipping is one reduction.

Parameters are laid out in *reverse* registration order, which is roughly
the order autograd finishes their gradients (heads first, input layer
last), so DP buckets become ready front-to-back.
Every segment starts on a 64-element (256 B) boundary so per-parameter
views stay 16-B aligned for vector loads.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Tuple

import torch

ALIGN = 64


class FlatArena:
    def __init__(self, params: Iterable[torch.nn.Parameter], device=None, reverse: bool = True):
        plist = [p for p in params if p.requires_grad]
        seen, uniq = set(), []
        for p in plist:
            if id(p) not in seen:
                seen.add(id(p))
                uniq.append(p)
        self.params: List[torch.nn.Parameter] = uniq[::-1] if reverse else uniq
        if not self.params:
            raise ValueError("FlatArena needs at least one trainable parameter")
        device = device or self.params[0].device
        self.offsets: List[Tuple[int, int]] = []
        off = 0
        for p in self.params:
            n = p.numel()
            self.offsets.append((off, n))
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        self.data = torch.zeros(off, dtype=torch.float32, device=device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=device)
        with torch.no_grad():
            for p, (o, n) in zip(self.params, self.offsets):
                self.data[o:o + n].copy_(p.detach().reshape(-1).float())
                p.data = self.data[o:o + n].view(p.shape)
                p._pbx_arena = True  # fused backward kernels may accumulate into p.grad directly
        self.attach_grads()

    def attach_grads(self) -> None:
        for p, (o, n) in zip(self.params, self.offsets):
            p.grad = self.grad[o:o + n].view(p.shape)

    def grads_attached(self) -> bool:
        base, es = self.grad.data_ptr(), self.grad.element_size()
        for p, (o, _) in zip(self.params, self.offsets):
            g = p.grad
            if g is None or g.data_ptr() != base + o * es:
                return False
        return True

    def zero_grad(self) -> None:
        if not self.grads_attached():
            self.attach_grads()
        if self.grad.is_cuda:
            from ..ops import _lib
            if _lib.available():
                # in-tree fill: the step runs no PyTorch-native kernel
                _lib.call("pbx_fill_flat", self.grad.data_ptr(), self.grad.numel(), 0.0, _lib.stream_ptr(self.grad.device))
                return
        self.grad.zero_()

    def attach_bf16_shadow(self, shadow: torch.Tensor) -> None:
        """Point every parameter's ``_pbx_bf16`` at its segment of a bf16 mirror of the arena that
        the fused optimizer rewrites on each update, so forward/backward GEMMs read bf16 weights
        without a cast launch per use.  A parameter written outside the optimizer (``p.copy_``,
        ``load_state_dict``) bumps its version counter and its segment is refreshed on next use
        (:func:`ops.global_track.bf16_of`)."""
        if shadow.numel() != self.numel or shadow.dtype != torch.bfloat16:
            raise ValueError("shadow must be a bf16 tensor with the arena's element count")
        for p, (o, n) in zip(self.params, self.offsets):
            p._pbx_bf16 = shadow[o:o + n].view(p.shape)
            p._pbx_bf16_ver = p._version

    def invalidate_bf16_shadow(self) -> None:
        """Force a refresh of every bf16 mirror on next use (after writes that bypass autograd's
        version counter, e.g. a collective broadcast into ``arena.data``)."""
        invalidate_bf16_mirrors(self.params)

    def param_index(self) -> Dict[int, int]:
        return {id(p): i for i, p in enumerate(self.params)}

    def segment(self, i: int) -> Tuple[int, int]:
        return self.offsets[i]


def invalidate_bf16_mirrors(params: Iterable[torch.Tensor]) -> None:
    for p in params:
        if getattr(p, "_pbx_bf16", None) is not None:
            p._pbx_bf16_ver = -1


# --- direct gradient writes ---------------------------------------------------------------------
# Fused backward kernels (ops.local_track) accumulate parameter gradients straight into the arena
# ``.grad`` views instead of returning them to autograd (which would launch one add kernel per
# parameter).  AccumulateGrad -- and with it ``post_accumulate_grad`` hooks -- then never runs for
# those parameters, so consumers that track gradient readiness (the DP bucketer) subscribe here.
_grad_ready_listeners = []


def add_grad_ready_listener(fn) -> None:
    _grad_ready_listeners.append(fn)


def remove_grad_ready_listener(fn) -> None:
    if fn in _grad_ready_listeners:
        _grad_ready_listeners.remove(fn)


def notify_grads_ready(params) -> None:
    for fn in list(_grad_ready_listeners):
        fn(params)
