"""Bucketed, backward-overlapped gradient all-reduce over the flat grad arena.

Design for 8x MI355X on xGMI: each GPU has 7 point-to-point
links (~153 GB/s each); a ring all-reduce is per-link bound, so throughput
needs (a) messages big enough to amortise RCCL's per-call latency and fill
its channels and (b) enough buckets to overlap with the 6-block backward.
The gradient payload is ~65-70 MB fp32; the default 8 MB buckets give ~9
collectives per step.

* Buckets are contiguous slices of :class:`~..train.arena.FlatArena.grad`,
  so RCCL reduces in place with no pack/unpack copies.
* The arena stores parameters in reverse registration order, which is the
  order autograd finishes them (GO head first, global input layer last), so
  buckets complete front-to-back; each parameter's
  ``post_accumulate_grad_hook`` counts down its bucket, and buckets are
  launched strictly in index order (every rank issues the same collective
  sequence) as soon as they are complete, during the rest of backward.
* Transport: on the nccl (RCCL) backend the buckets go through a direct RCCL communicator
  (:mod:`.rccl`) whose ``ncclAllReduce`` is enqueued on the conv weight-gradient stream that produces
  each bucket's last gradients -- no process-group stream and no event pair per bucket (the process
  group's extra stream shared a hardware queue with the step's streams: +3.7 ms on a forced 1-rank step,
  ``profiles/r5/dp_host_and_flags.txt``).  gloo groups (CPU tests) and ``PBX_DP_COMM=torch`` use
  ``torch.distributed.all_reduce``.
* ``SUM`` reduction; the 1/world factor is folded into the fused Adam
  (``FusedAdam.grad_scale``) instead of an extra pass.
* :meth:`finish_and_step` (the training step's default with the fused Adam) hides the optimizer
  behind the exposed tail: the buckets whose gradients are final only after backward (the global input
  layer + block 0, ~20 MB) are still on the wire when the Adam update of every other bucket runs on the
  compute stream; only the tail buckets' update trails their all-reduce.
* Non-finite steps are skipped group-wide, decided BEFORE any update: every bucket's LOCAL gradients
  are tested on the collective stream right before its all-reduce (one small kernel pair beside the
  backward), with a conservative bound -- an element counts as bad when it is NaN / Inf or
  ``|g| >= FLT_MAX / world``, so no sum of the ranks' accepted values can overflow fp32 -- and the
  per-rank flag goes through one 4-byte MAX all-reduce queued ahead of the tail buckets.  Every rank
  then skips or commits the whole step together (no partially applied step).
* ``comm_dtype=torch.bfloat16`` reduces every bucket through a bf16 copy (half the xGMI bytes,
  bf16-rounded gradient sums); the default is fp32.
"""
from __future__ import annotations

import contextlib
import os
import warnings
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import streams
from . import rccl
from ..train.arena import FlatArena, add_grad_ready_listener, remove_grad_ready_listener

FLT_MAX = 3.4028234663852886e38


class BucketedAllReduce:
    def __init__(self, arena: FlatArena, bucket_mb: float = 8.0, process_group=None,
                 comm_dtype: torch.dtype = torch.float32, force: bool = False):
        """``force`` runs the hooks and collectives even on a 1-rank group (tests of the stream
        ordering on a single GPU)."""
        self.arena = arena
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.comm_dtype = comm_dtype
        limit = int(bucket_mb * 1024 * 1024 / 4)
        # bucket = [start, end) in arena elements, built on parameter boundaries
        self.buckets: List[List[int]] = []
        self.param_bucket: List[int] = []
        start, cur_end = None, 0
        for i, (o, n) in enumerate(arena.offsets):
            if start is None:
                start = o
            seg_end = arena.offsets[i + 1][0] if i + 1 < len(arena.offsets) else arena.numel
            self.param_bucket.append(len(self.buckets))
            cur_end = seg_end
            if cur_end - start >= limit:
                self.buckets.append([start, cur_end])
                start = None
        if start is not None:
            if self.buckets and cur_end - start < limit // 4:
                # a small remainder (the embedding / input-layer bias, last to finish) joins the last
                # bucket: one collective instead of two latency-bound ones at the exposed end of backward
                self.buckets[-1][1] = cur_end
                for i in range(len(self.param_bucket)):
                    if self.param_bucket[i] == len(self.buckets):
                        self.param_bucket[i] = len(self.buckets) - 1
            else:
                self.buckets.append([start, cur_end])
        self.bucket_nparams = [0] * len(self.buckets)
        for b in self.param_bucket:
            self.bucket_nparams[b] += 1
        self._pending = list(self.bucket_nparams)
        # a parameter is counted ONCE per step: fused backward kernels write some gradients in place
        # and announce them (_on_direct_grads), and autograd still runs those parameters'
        # AccumulateGrad node (with no gradient) and its post-accumulate hook afterwards -- counting
        # both launched buckets before their last gradient was written
        self._ready = [False] * len(arena.params)
        self._works: List[Optional[object]] = [None] * len(self.buckets)
        # overlapped optimizer (finish_and_step).  PBX_DP_OVERLAP_OPT=0: finish() + one whole-arena update
        # after every all-reduce (A/B knob)
        self.overlap_optimizer = os.environ.get("PBX_DP_OVERLAP_OPT", "1") != "0"
        self.track_nonfinite = False
        # bad element: NaN / Inf, or so large that the sum over the ranks could overflow fp32
        self.nonfinite_bound = FLT_MAX / max(1, self.world)
        self._flag: Optional[torch.Tensor] = None       # int32 [1]: this rank's flag, then the group MAX
        self._flag_fresh = True
        self._flag_work = None
        self._nf_ws: Optional[torch.Tensor] = None
        self._tmp: List[Optional[torch.Tensor]] = [None] * len(self.buckets)
        self._next = 0
        self._hooks = []
        self.enabled = self.world > 1 or (force and dist.is_initialized())
        self._index = {id(p): i for i, p in enumerate(arena.params)}
        self.comm: Optional[rccl.Communicator] = None
        self._ev_head: Optional[torch.cuda.Event] = None
        self._ev_tail: Optional[torch.cuda.Event] = None
        self._evs = None
        if self.enabled:
            if arena.grad.is_cuda and rccl.wanted(process_group):
                try:
                    self.comm = rccl.Communicator(process_group, device=arena.grad.device)
                except Exception as e:       # noqa: BLE001 - keep training on the process-group path
                    warnings.warn(f"direct RCCL communicator unavailable ({e}); using torch.distributed")
                    self.comm = None
            for i, p in enumerate(arena.params):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
            add_grad_ready_listener(self._on_direct_grads)

    @property
    def transport(self) -> str:
        return "rccl-direct" if self.comm is not None else ("torch.distributed" if self.enabled else "none")

    # --------------------------------------------------------------------------------
    def _mark(self, i: int) -> None:
        if not self._ready[i]:
            self._ready[i] = True
            self._pending[self.param_bucket[i]] -= 1

    def _make_hook(self, idx: int):
        def hook(_p):
            self._mark(idx)
            self._launch_ready()
        return hook

    def _on_direct_grads(self, params) -> None:
        """Gradients written in place by a fused backward kernel (enqueued on the current or an aux
        stream; the collective is ordered behind both)."""
        for p in params:
            i = self._index.get(id(p))
            if i is not None:
                self._mark(i)
        self._launch_ready()

    def _local_flag(self, view: torch.Tensor) -> None:
        """flag |= 1 when this rank's gradients in ``view`` hold a NaN / Inf or an element at or above
        :attr:`nonfinite_bound` (before the in-place all-reduce overwrites them), on the current stream
        (the one the collective is ordered on).  The first test of a step overwrites the flag."""
        if self._flag is None or self._flag.device != view.device:
            self._flag = torch.zeros(1, dtype=torch.int32, device=view.device)
        acc = 0 if self._flag_fresh else 1
        self._flag_fresh = False
        if view.is_cuda:
            from ..ops import _lib
            if self._nf_ws is None:
                self._nf_ws = torch.empty(1024, dtype=torch.int32, device=view.device)
            _lib.call("pbx_nonfinite_flag", view.data_ptr(), view.numel(), self._nf_ws.data_ptr(),
                      self._flag.data_ptr(), self.nonfinite_bound, acc, _lib.stream_ptr(view.device))
        else:
            bad = 1 if view.numel() and not bool((view.abs() < self.nonfinite_bound).all()) else 0
            self._flag[0] = bad if acc == 0 else max(int(self._flag[0]), bad)

    def _all_reduce(self, t: torch.Tensor, op: str = "sum"):
        """Enqueue an in-place all-reduce of ``t`` behind the current stream's work; returns the work
        handle to wait for (None for the direct communicator: stream-ordered, see :meth:`_record`)."""
        if self.comm is not None:
            self.comm.all_reduce_(t, op)
            return None
        rop = dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM
        return dist.all_reduce(t, op=rop, group=self.pg, async_op=True)

    def _record(self, i: int) -> Optional[torch.cuda.Event]:
        """Event ``i`` (0: head, 1: tail; cached, re-recorded every step) after the work enqueued so far
        on the current (collective) stream."""
        if self.comm is None:
            return None
        if self._evs is None:
            self._evs = (torch.cuda.Event(), torch.cuda.Event())
        self._evs[i].record()
        return self._evs[i]

    def _launch(self, b: int, flag: bool = True) -> None:
        s, e = self.buckets[b]
        view = self.arena.grad[s:e]
        dt = self.comm_dtype
        # a bucket may hold conv weight gradients still being produced on the aux stream
        # (ops/streams.py): enqueue the collective behind both streams without stalling this one
        ctx = streams.collective_stream(view.device) if view.is_cuda else contextlib.nullcontext()
        with ctx:
            if flag and self.track_nonfinite:
                self._local_flag(view)
            if dt != torch.float32:
                tmp = view.to(dt)
                self._tmp[b] = tmp
                self._works[b] = self._all_reduce(tmp)
            else:
                self._works[b] = self._all_reduce(view)

    def _flag_reduce_and_launch_rest(self) -> None:
        """Local flags of the buckets not launched yet, the group-wide MAX of the flag (4 bytes, queued
        ahead of them), then those buckets' all-reduces."""
        rest = range(self._next, len(self.buckets))
        dev = self.arena.grad.device
        ctx = streams.collective_stream(dev) if self.arena.grad.is_cuda else contextlib.nullcontext()
        with ctx:
            for b in rest:
                s, e = self.buckets[b]
                self._local_flag(self.arena.grad[s:e])
            if self._flag is None:
                self._flag = torch.zeros(1, dtype=torch.int32, device=dev)
            self._flag_work = self._all_reduce(self._flag, "max")
            self._ev_head = self._record(0)         # head buckets and the group flag have landed
            for b in rest:
                self._launch(b, flag=False)
            self._ev_tail = self._record(1)
        self._next = len(self.buckets)

    def _land(self, b: int) -> None:
        """Current stream waits for bucket b's all-reduce (and copies a reduced bf16 bucket back)."""
        w = self._works[b]
        if w is not None:
            w.wait()
        if self._tmp[b] is not None:
            s, e = self.buckets[b]
            self.arena.grad[s:e].copy_(self._tmp[b])
            self._tmp[b] = None

    def _launch_ready(self) -> None:
        # overlapped optimizer step: the LAST bucket stays for finish_and_step, so the group-wide
        # non-finite flag's all-reduce is queued ahead of it and the update of buckets 0..n-2 runs
        # beside the last (largest: embedding + input layer) all-reduce instead of after it
        end = len(self.buckets) - (1 if self.track_nonfinite and len(self.buckets) > 1 else 0)
        while self._next < end and self._pending[self._next] <= 0:
            self._launch(self._next)
            self._next += 1

    def start_step(self) -> None:
        self._pending = list(self.bucket_nparams)
        self._ready = [False] * len(self._ready)
        self._next = 0
        self._works = [None] * len(self.buckets)
        self._flag_fresh = True
        self._ev_head = self._ev_tail = None

    def finish(self, average: bool = False) -> None:
        """Launch any bucket whose params got no gradient, then wait (stream-ordered)."""
        if not self.enabled:
            return
        if self.arena.grad.is_cuda:
            streams.join()
        for b in range(self._next, len(self.buckets)):
            self._launch(b)
        self._next = len(self.buckets)
        if self.arena.grad.is_cuda:
            streams.join_collectives(self.arena.grad.device)   # direct communicator: its stream
        for b in range(len(self.buckets)):
            self._land(b)
        if average:
            self.arena.grad.div_(self.world)
        self.track_nonfinite = False
        self.start_step()

    def finish_and_step(self, opt, skip_nonfinite: bool = True) -> None:
        """End of backward for the fused Adam: buckets 0..n-2 are updated as soon as the group-wide
        non-finite flag (queued ahead of the last bucket) has landed, beside the last bucket's
        all-reduce; the last bucket's update follows its all-reduce.  Bitwise the same parameters as
        :meth:`finish` + a whole-arena ``opt.step()`` (Adam is element-wise).  Call
        :meth:`begin_overlapped_step` before backward (the buckets launched during backward test their
        local gradients then)."""
        if not self.enabled:
            if skip_nonfinite:
                opt.set_nonfinite_skip()
            opt.step()
            return
        if not self.track_nonfinite and self._next > 0:
            raise RuntimeError("finish_and_step: begin_overlapped_step() was not called before backward")
        cuda = self.arena.grad.is_cuda
        if cuda:
            streams.join()
        split_b = self._next
        self._flag_reduce_and_launch_rest()
        cur = torch.cuda.current_stream(self.arena.grad.device) if cuda else None
        if self._ev_head is not None:
            cur.wait_event(self._ev_head)
        for b in range(split_b):
            self._land(b)
        if self._flag_work is not None:
            self._flag_work.wait()
        split = self.buckets[split_b][0] if split_b < len(self.buckets) else self.arena.numel
        # every rank holds the same group-wide flag: the whole step is skipped or committed together
        opt.skip_flag = self._flag if skip_nonfinite else None
        opt.begin_step()
        opt.step_range(0, split)              # beside the tail buckets' all-reduce
        if self._ev_tail is not None:
            cur.wait_event(self._ev_tail)
        for b in range(split_b, len(self.buckets)):
            self._land(b)
        opt.step_range(split, self.arena.numel)
        if cuda:
            streams.join_collectives(self.arena.grad.device)
        self.track_nonfinite = False
        self._flag_work = None
        self.start_step()

    def begin_overlapped_step(self) -> None:
        """The coming backward's buckets carry local non-finite flags (for :meth:`finish_and_step`)."""
        self.track_nonfinite = self.enabled
        self._flag_fresh = True

    def broadcast_parameters(self, module: Optional[torch.nn.Module] = None, src: int = 0) -> None:
        if not self.enabled:
            return
        dist.broadcast(self.arena.data, src, group=self.pg)
        self.arena.invalidate_bf16_shadow()
        if module is not None:
            for buf in module.buffers():
                dist.broadcast(buf.data, src, group=self.pg)

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
        remove_grad_ready_listener(self._on_direct_grads)

    def close(self) -> None:
        """Remove the hooks and release the direct communicator (before the process group goes)."""
        self.remove_hooks()
        if self.comm is not None:
            self.comm.close()
            self.comm = None
