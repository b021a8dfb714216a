"""Side-stream execution of off-critical-path backward work (the conv weight gradients).

In one block's backward the conv weight gradient (``pbx_wgrad`` + its slab reduction, ~1 ms of a
5.8 ms paper-config step) depends only on ``dpre`` and the block input, and nothing else in the
backward reads its result: the next kernels on the critical path (the previous block's attention /
LayerNorm / conv-dgrad chain) need only ``dx``.  Issuing it on a second HIP stream lets the
hardware run its MFMA-bound waves beside the bandwidth-bound LayerNorm/attention kernels.

Protocol (also valid under hipGraph capture, where the fork/join becomes graph edges):

* :func:`launch` makes the aux stream wait for the current stream, runs ``fn`` under the aux
  stream (allocations inside ``fn`` belong to the aux stream's pool) and keeps ``keep`` tensors
  alive until the join, so the caching allocator cannot hand their memory to the main stream while
  the aux stream still reads them.
* :func:`join` makes the main stream wait for the aux stream and drops the kept tensors.  It is
  queued as an autograd end-of-backward callback, called again by :class:`..train.step.PretrainStep`
  before the optimizer, and :func:`collective_stream` lets the DP reducer order a bucket's all-reduce
  after the aux-stream gradients that bucket contains.
"""
from __future__ import annotations

import os
from contextlib import contextmanager
from typing import Callable, Dict, List, Optional

import torch

ENABLED = os.environ.get("PBX_AUX_STREAM", "1") != "0"

_streams: Dict[int, torch.cuda.Stream] = {}
_pending: Dict[int, List[torch.Tensor]] = {}
_main: Dict[int, torch.cuda.Stream] = {}
_callback_queued = {"v": False}


def _aux(device: torch.device) -> torch.cuda.Stream:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _streams.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=idx)
        _streams[idx] = s
    return s


def active(device: Optional[torch.device] = None) -> bool:
    if device is None:
        return any(_pending.values())
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return bool(_pending.get(idx))


def launch(device: torch.device, fn: Callable[[], Optional[List[torch.Tensor]]], keep: List[torch.Tensor]) -> None:
    """Run ``fn`` (kernel launches) on the aux stream of ``device`` after the current stream's work.
    ``keep`` and the tensors ``fn`` returns (its scratch) stay referenced until :func:`join`: an
    aux-pool block freed earlier could be handed to a main-stream writer while aux kernels still
    use it."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    main = torch.cuda.current_stream(idx)
    aux = _aux(device)
    aux.wait_stream(main)
    with torch.cuda.stream(aux):
        scratch = fn() or []
    _pending.setdefault(idx, []).extend(list(keep) + list(scratch))
    _main[idx] = main
    if not _callback_queued["v"]:
        try:
            torch.autograd.Variable._execution_engine.queue_callback(join)
            _callback_queued["v"] = True
        except RuntimeError:          # not inside a backward pass: the caller joins explicitly
            pass


def join() -> None:
    """Main stream(s) wait for the aux stream(s); release the tensors kept for them."""
    _callback_queued["v"] = False
    for idx, keep in list(_pending.items()):
        if not keep:
            continue
        main = _main.get(idx) or torch.cuda.current_stream(idx)
        main.wait_stream(_streams[idx])
        keep.clear()


@contextmanager
def collective_stream(device: torch.device):
    """Context for issuing a collective over gradients that may include aux-stream results: the
    collective is enqueued behind both the current stream's and the aux stream's work, without
    making the current stream wait."""
    if not active(device):
        yield
        return
    aux = _aux(device)
    aux.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(aux):
        yield
