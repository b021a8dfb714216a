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
  sequence) as soon as they are complete — overlapping with the rest of
  backward on RCCL's own stream.
* ``SUM`` reduction; the 1/world factor is folded into the fused Adam
  (``FusedAdam.grad_scale``) instead of an extra pass.
* :meth:`finish_and_step` (the training step's default with the fused Adam) hides the optimizer
  behind the exposed tail: the buckets whose gradients are final only after backward (the global input
  layer + block 0, ~20 MB) are still on the wire when the Adam update of every other bucket runs on the
  compute stream; only the tail buckets' update trails their all-reduce.  The group-wide non-finite
  decision is taken BEFORE any update: the tail buckets' local gradients are tested when they are
  launched and one 4-byte MAX all-reduce of those flags is queued ahead of them; the head buckets are
  tested after their all-reduce (a NaN / Inf on any rank survives the sum, and the reduced values are
  identical on every rank, so no extra collective), so every rank skips or commits every bucket
  together.  (Testing each head bucket's local gradients as it was launched put a kernel and two
  cross-stream waits per bucket on the communication stream during backward: -48 % on a forced 1-rank
  RCCL step, profiles/r5/dp_host_and_flags.txt.)  A sum of finite per-rank gradients that overflows fp32
  skips the whole step when it is in the head buckets, and the tail update (with the head already
  committed) when it appears only in the tail -- no Inf / NaN ever reaches the parameters.
* ``comm_dtype=torch.bfloat16`` reduces every bucket through a bf16 copy (half the xGMI bytes,
  bf16-rounded gradient sums); the default is fp32.  (A bf16 reduction of only the last, exposed
  bucket -- the 18 MB global input layer -- was an unmeasured option and has been removed: no
  multi-rank run on this pool could show whether its saving beats the two conversion passes.)
"""
from __future__ import annotations

import contextlib
import os
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import streams
from ..train.arena import FlatArena, add_grad_ready_listener, remove_grad_ready_listener


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
        # overlapped optimizer (finish_and_step): per-bucket local non-finite flags, group-wide OR.
        # PBX_DP_OVERLAP_OPT=0: finish() + one whole-arena update after every all-reduce (A/B knob)
        self.overlap_optimizer = os.environ.get("PBX_DP_OVERLAP_OPT", "1") != "0"
        self.track_nonfinite = False
        self._flags: Optional[torch.Tensor] = None
        self._gflag: Optional[torch.Tensor] = None
        self._flag_work = None
        self._nf_ws: Optional[torch.Tensor] = None
        self._tmp: List[Optional[torch.Tensor]] = [None] * len(self.buckets)
        self._next = 0
        self._hooks = []
        self.enabled = self.world > 1 or (force and dist.is_initialized())
        self._index = {id(p): i for i, p in enumerate(arena.params)}
        if self.enabled:
            for i, p in enumerate(arena.params):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
            add_grad_ready_listener(self._on_direct_grads)

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

    def _local_flag(self, b: int, view: torch.Tensor) -> None:
        """flags[b] = 1 when this rank's gradients of bucket b hold a NaN / Inf (before the in-place
        all-reduce overwrites them), on the stream the collective is ordered on."""
        if self._flags is None or self._flags.device != view.device:
            self._flags = torch.zeros(len(self.buckets), dtype=torch.int32, device=view.device)
        if view.is_cuda:
            from ..ops import _lib
            if self._nf_ws is None:
                self._nf_ws = torch.empty(1024, dtype=torch.int32, device=view.device)
            _lib.call("pbx_nonfinite_flag", view.data_ptr(), view.numel(), self._nf_ws.data_ptr(),
                      self._flags[b:].data_ptr(), _lib.stream_ptr(view.device))
        else:
            bad = not bool(torch.isfinite(torch.dot(view, torch.zeros_like(view))))
            self._flags[b] = 1 if bad else 0

    def _launch(self, b: int, flag_done: bool = False) -> None:
        s, e = self.buckets[b]
        view = self.arena.grad[s:e]
        dt = self.comm_dtype
        # a bucket may hold conv weight gradients still being produced on the aux stream
        # (ops/streams.py): enqueue the collective behind both streams without stalling this one
        ctx = streams.collective_stream(view.device) if view.is_cuda else contextlib.nullcontext()
        with ctx:
            # no local non-finite flag for a bucket launched during backward: finish_and_step checks the
            # REDUCED head gradients (a NaN / Inf on any rank survives the sum), so only the buckets held
            # for the end need local flags (their update must be decided before their all-reduce lands)
            if dt != torch.float32:
                tmp = view.to(dt)
                self._tmp[b] = tmp
                self._works[b] = dist.all_reduce(tmp, group=self.pg, async_op=True)
            else:
                self._works[b] = dist.all_reduce(view, group=self.pg, async_op=True)

    def _post_flag(self, start: int, end: int) -> torch.Tensor:
        """int32 [1] device flag: 1 when the (reduced) arena gradients [start, end) hold a NaN / Inf."""
        view = self.arena.grad[start:end]
        if view.is_cuda:
            from ..ops import _lib
            ws = torch.empty(1025, dtype=torch.int32, device=view.device)
            if view.numel() == 0:
                return ws[1024:].zero_()
            _lib.call("pbx_nonfinite_flag", view.data_ptr(), view.numel(), ws.data_ptr(), ws[1024:].data_ptr(),
                      _lib.stream_ptr(view.device))
            return ws[1024:]
        bad = view.numel() > 0 and not bool(torch.isfinite(torch.dot(view, torch.zeros_like(view))))
        return torch.tensor([1 if bad else 0], dtype=torch.int32, device=view.device)

    def _flag_reduce_and_launch_rest(self) -> None:
        """Local flags of the buckets not launched yet, the group-wide MAX of every bucket's flag (4 bytes,
        queued ahead), then those buckets' all-reduces."""
        rest = range(self._next, len(self.buckets))
        dev = self.arena.grad.device
        ctx = streams.collective_stream(dev) if self.arena.grad.is_cuda else contextlib.nullcontext()
        with ctx:
            self._flags.zero_()
            for b in rest:
                s, e = self.buckets[b]
                self._local_flag(b, self.arena.grad[s:e])
            self._gflag = self._flags.amax().reshape(1)
            self._flag_work = dist.all_reduce(self._gflag, op=dist.ReduceOp.MAX, group=self.pg, async_op=True)
        for b in rest:
            self._launch(b, flag_done=True)
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

    def finish(self, average: bool = False) -> None:
        """Launch any bucket whose params got no gradient, then wait (stream-ordered)."""
        if not self.enabled:
            return
        if self.arena.grad.is_cuda:
            streams.join()
        for b in range(self._next, len(self.buckets)):
            self._launch(b)
        self._next = len(self.buckets)
        for b in range(len(self.buckets)):
            self._land(b)
        if self.arena.grad.is_cuda:
            streams.join_collectives(self.arena.grad.device)
        if average:
            self.arena.grad.div_(self.world)
        self.start_step()

    def finish_and_step(self, opt, skip_nonfinite: bool = True) -> None:
        """End of backward for the fused Adam: buckets 0..n-2 are updated as soon as the group-wide
        non-finite flag (queued ahead of the last bucket) has landed, beside the last bucket's
        all-reduce; the last bucket's update follows its all-reduce.  Bitwise the same parameters as
        :meth:`finish` + a whole-arena ``opt.step()`` (Adam is element-wise).  Call
        :meth:`begin_overlapped_step` before backward."""
        if not self.enabled:
            if skip_nonfinite:
                opt.set_nonfinite_skip()
            opt.step()
            return
        if self.arena.grad.is_cuda:
            streams.join()
        if self._flags is None:
            self._flags = torch.zeros(len(self.buckets), dtype=torch.int32, device=self.arena.grad.device)
        # the exposed tail: buckets whose gradients were not final during backward (launched only now)
        # (all of them launched already: the update waits only for the flag, queued behind them)
        split_b = self._next
        self._flag_reduce_and_launch_rest()
        for b in range(split_b):
            self._land(b)
        self._flag_work.wait()
        split = self.buckets[split_b][0] if split_b < len(self.buckets) else self.arena.numel
        skip = None
        if skip_nonfinite:
            # local flags (group OR) + the REDUCED head gradients: finite per-rank gradients whose sum
            # overflows are caught too; the reduced values are identical on every rank, so every rank
            # takes the same decision without another collective
            skip = torch.maximum(self._gflag, self._post_flag(0, split))
        opt.skip_flag = skip
        opt.begin_step()
        opt.step_range(0, split)              # beside the tail buckets' all-reduce
        for b in range(split_b, len(self.buckets)):
            self._land(b)
        if split < self.arena.numel:
            if skip_nonfinite:
                # a sum that overflows only in the tail is known only now: the tail update is skipped
                # (the head's was already committed), so no Inf / NaN ever reaches the parameters
                opt.skip_flag = torch.maximum(skip, self._post_flag(split, self.arena.numel))
            opt.step_range(split, self.arena.numel)
        if self.arena.grad.is_cuda:
            streams.join_collectives(self.arena.grad.device)
        self.track_nonfinite = False
        self._flag_work = None
        self.start_step()

    def begin_overlapped_step(self) -> None:
        """The coming backward's buckets carry local non-finite flags (for :meth:`finish_and_step`)."""
        self.track_nonfinite = self.enabled

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
