"""Side-stream execution of off-critical-path backward work.

Two pieces of one block's backward do not feed the critical path directly:

* ``wgrad``  - the conv weight gradient (``pbx_wgrad`` + slab reduction, ~1 ms of a 5 ms
  paper-config step): only the optimizer and the DP all-reduce read it;
* ``head`` / ``ann`` - the GO head's forward beside the local head, the input layer's backward beside
  the first block's conv data gradient (ops/global_track.py).

(Rounds 2-4 also measured the conv data gradient and the global-track backward on streams of their own:
1.9 % and 1 % slower -- their kernels only found CUs as the critical-path kernels drained; removed.)

Issuing them on their own HIP streams lets the hardware run them beside the main-stream kernels.
Protocol (eager and under hipGraph capture, where fork/join become graph edges):

* :func:`on_aux` makes the named aux stream wait for the current stream (or for an earlier
  :func:`fork` point of it) and runs the body on it;
  every tensor the body reads that was allocated by the main stream, and every output another
  stream consumes, is kept referenced until :func:`join` (the caching allocator could otherwise
  hand the memory to another stream's writer while the aux kernels still use it).
* :func:`mark_ready` notes which aux stream produced a tensor; a consumer on another stream calls
  :func:`wait_ready` before reading it (a stream-level wait: work already enqueued on the consumer
  stream keeps overlapping).
* :func:`join` makes the main stream wait for every aux stream (queued as an autograd
  end-of-backward callback and called by :class:`..train.step.PretrainStep`), and
  :func:`collective_stream` orders a DP all-reduce behind the main stream and every aux stream, on the
  weight-gradient stream.
"""
from __future__ import annotations

import os
from contextlib import contextmanager
from typing import Dict, Iterable, List, Optional, Tuple

import torch

ENABLED = os.environ.get("PBX_AUX_STREAM", "1") != "0"            # conv weight gradient
_streams: Dict[Tuple[int, str], torch.cuda.Stream] = {}
_pending: Dict[int, List[torch.Tensor]] = {}
_used: Dict[int, set] = {}
_main: Dict[int, torch.cuda.Stream] = {}
_ready: Dict[int, Tuple[int, str]] = {}
_callback_queued = {"v": False}


def _idx(device: torch.device) -> int:
    return device.index if device.index is not None else torch.cuda.current_device()


def _aux(device: torch.device, name: str = "wgrad") -> torch.cuda.Stream:
    key = (_idx(device), name)
    s = _streams.get(key)
    if s is None:
        s = torch.cuda.Stream(device=key[0])
        _streams[key] = s
    return s


def active(device: Optional[torch.device] = None) -> bool:
    if device is None:
        return any(_pending.values())
    return bool(_pending.get(_idx(device)))


def queue_join() -> None:
    """Queue :func:`join` at the end of the running backward pass (no-op outside one)."""
    _queue_join()


def _queue_join() -> None:
    if not _callback_queued["v"]:
        try:
            torch.autograd.Variable._execution_engine.queue_callback(join)
            _callback_queued["v"] = True
        except RuntimeError:          # not inside a backward pass: the caller joins explicitly
            pass


class _AuxScope:
    def __init__(self, idx: int):
        self.idx = idx

    def keep(self, *tensors) -> None:
        _pending.setdefault(self.idx, []).extend(t for t in tensors if isinstance(t, torch.Tensor))


_forked: Dict[Tuple[int, str], bool] = {}


_events: Dict[Tuple[int, int], torch.cuda.Event] = {}
# Under hipGraph capture a fork whose aux body starts at the main stream's current tail makes that tail
# node have two children, and the graph executor continues a node's queue with its FIRST child in
# capture order -- the aux body (e.g. the conv weight gradient) would take the main chain's queue and
# the critical path would wait behind it.  An empty main-stream kernel is captured before the aux body so
# the main chain is the first child (tests/test_graph_step.py).


def _wait(dst: torch.cuda.Stream, src: torch.cuda.Stream) -> None:
    """``dst`` waits for the work enqueued on ``src`` so far.  ``Stream.wait_stream`` creates a new
    event per call (~20 such hand-offs per step); a wait binds to the event's latest record at the
    time it is enqueued, so one cached event per (dst, src) pair is reused."""
    key = (dst.cuda_stream, src.cuda_stream)
    ev = _events.get(key)
    if ev is None:
        ev = _events[key] = torch.cuda.Event()
    ev.record(src)
    dst.wait_event(ev)


def fork(device: torch.device, name: str) -> None:
    """Make aux stream ``name`` wait for the current stream's work enqueued SO FAR; the next
    :func:`on_aux` on it starts from this point instead of the current stream's later tail (the
    main stream can enqueue more work that the aux body does not need)."""
    _wait(_aux(device, name), torch.cuda.current_stream(_idx(device)))
    _forked[(_idx(device), name)] = True


def forked(device: torch.device, name: str) -> bool:
    """A :func:`fork` of aux stream ``name`` is pending (the next :func:`on_aux` starts from it)."""
    return _forked.get((_idx(device), name), False)


def cancel_fork(device: torch.device, name: str) -> None:
    _forked.pop((_idx(device), name), None)


@contextmanager
def on_aux(device: torch.device, name: str, keep: Iterable[torch.Tensor] = ()):
    """Run the body on aux stream ``name`` of ``device`` after the current stream's work (or after
    the pending :func:`fork` point of that stream)."""
    idx = _idx(device)
    main = torch.cuda.current_stream(idx)
    aux = _aux(device, name)
    if not _forked.pop((idx, name), False):
        _wait(aux, main)
        if torch.cuda.is_current_stream_capturing():
            from . import _lib
            _lib.call("pbx_noop", main.cuda_stream)
    scope = _AuxScope(idx)
    scope.keep(*keep)
    _used.setdefault(idx, set()).add(name)
    _main[idx] = main
    # set_stream in place of the torch.cuda.stream context (the step enters ~20 of these scopes;
    # the context manager's device bookkeeping cost ~20 us of host time each)
    torch.cuda.set_stream(aux)
    try:
        yield scope
    finally:
        torch.cuda.set_stream(main)
    _queue_join()


def launch(device: torch.device, fn, keep: List[torch.Tensor], name: str = "wgrad") -> None:
    """Run ``fn`` (kernel launches) on aux stream ``name``; ``keep`` and the tensors ``fn`` returns
    (its scratch) stay referenced until :func:`join`."""
    with on_aux(device, name, keep) as scope:
        scope.keep(*(fn() or []))


def mark_ready(device: torch.device, name: str, tensors: Iterable[torch.Tensor]) -> None:
    """Record that ``tensors`` are outputs of aux stream ``name`` (complete once the work enqueued
    on it so far has run)."""
    for t in tensors:
        if isinstance(t, torch.Tensor):
            _ready[t.data_ptr()] = (_idx(device), name)


def chain(device: torch.device, dst: str, src: str) -> None:
    """Aux stream ``dst`` waits for the work enqueued on aux stream ``src`` so far."""
    _wait(_aux(device, dst), _aux(device, src))
    _used.setdefault(_idx(device), set()).add(dst)


def wait_for(device: torch.device, name: str) -> None:
    """Current stream waits for the work enqueued on aux stream ``name`` so far."""
    _wait(torch.cuda.current_stream(_idx(device)), _aux(device, name))


def wait_ready(*tensors) -> None:
    """Current stream waits for the aux-stream producer of any of ``tensors`` (no-op otherwise).
    The wait is on the producer stream's current tail (``wait_stream``: an event recorded and
    waited at once, which stays valid under hipGraph capture; an event recorded during capture
    and waited later would become a graph node owning a soon-destroyed event)."""
    for t in tensors:
        if isinstance(t, torch.Tensor):
            key = _ready.pop(t.data_ptr(), None)
            if key is not None:
                cur = torch.cuda.current_stream(t.device)
                if cur != _streams[key]:      # a stream waiting on itself is a no-op (and breaks graph capture)
                    _wait(cur, _streams[key])


def join() -> None:
    """Main stream(s) wait for every aux stream; release the tensors kept for them."""
    _callback_queued["v"] = False
    for idx, keep in list(_pending.items()):
        if not keep and not _used.get(idx):
            continue
        main = _main.get(idx) or torch.cuda.current_stream(idx)
        for name in _used.get(idx, ()):
            _wait(main, _streams[(idx, name)])
        keep.clear()
        _used[idx] = set()
    _ready.clear()
    _forked.clear()


@contextmanager
def collective_stream(device: torch.device):
    """Context for a collective over gradients that may include aux-stream results, without making the
    main stream wait.  It is enqueued on the conv weight-gradient stream (``wgrad``, which produces the
    bucket's last gradients) behind the main stream and every other aux stream in use.

    Why not a dedicated communication stream: HIP multiplexes streams onto GPU_MAX_HW_QUEUES hardware
    queues (4 on the pool), and a stream's wait on another stream's event is a barrier packet that stalls
    its whole hardware queue.  The communication stream shared the main stream's queue, so every bucket's
    wait for the weight-gradient stream stalled the critical path (~0.3 ms per bucket, -30 % on a forced
    1-rank RCCL step, profiles/r5/dp_host_and_flags.txt).  The weight-gradient stream lags the main stream,
    so its wait for the main stream is normally already satisfied, and its own queue is the one that
    would wait anyway."""
    idx = _idx(device)
    names = _used.get(idx)
    if not names:
        yield
        return
    host = _aux(device, "wgrad") if "wgrad" in names else _aux(device, "comm")
    _wait(host, torch.cuda.current_stream(idx))
    for name in names:
        other = _streams[(idx, name)]
        if other is not host:
            _wait(host, other)
    with torch.cuda.stream(host):
        yield


def join_collectives(device: torch.device) -> None:
    """Current stream waits for the streams :func:`collective_stream` enqueued on (the non-finite flag
    kernels; the collectives themselves are joined by ``work.wait()``).  Under hipGraph capture every stream
    forked into the capture must rejoin the capturing stream before the capture ends."""
    cur = torch.cuda.current_stream(_idx(device))
    for name in ("comm", "wgrad"):
        s = _streams.get((_idx(device), name))
        if s is not None:
            _wait(cur, s)


