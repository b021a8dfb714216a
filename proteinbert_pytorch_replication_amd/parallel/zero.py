"""ZeRO-1: Adam state sharded over the data-parallel group ("ZeRO / FSDP / optimizer
sharding" row — optional for this model, provided for large DP degrees and bigger configs).

Each rank keeps ``exp_avg`` / ``exp_avg_sq`` for one contiguous, ALIGN-rounded slice of the flat
parameter arena (``train/arena.py``) instead of all of it. ``step()`` is:

1. reduce-scatter of the flat gradient (SUM; the 1/world mean is folded into the Adam launch's
   ``grad_scale``) — each rank receives only its slice, i.e. half the bytes of an all-reduce;
2. the fused Adam launch (``pbx_adam_flat``, ``csrc/optim.hip``) on that slice only;
3. all-gather of the updated fp32 slices back into every rank's arena (+ bf16 mirror refresh).

Reduce-scatter + all-gather move the same bytes as one ring all-reduce over xGMI, so step time is
unchanged while optimizer memory drops by the DP degree. Use it *instead of*
:class:`~.ddp.BucketedAllReduce` (the collective happens at ``step()``, not overlapped with
backward). ``state_dict()`` gathers the full moments and has exactly ``torch.optim.Adam``'s format,
so checkpoints are interchangeable with :class:`~..train.optim.FusedAdam`. On gloo (CPU tests)
the reduce-scatter / all-gather are emulated with all-reduce / all_gather lists.
"""
from __future__ import annotations

from typing import Any, Dict, Optional

import torch
import torch.distributed as dist

from ..train.arena import ALIGN
from ..train.optim import FusedAdam, _hip_ok, adam_update_host, skip_requested


class ZeroFusedAdam(FusedAdam):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, process_group=None, **kw):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, **kw)
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        a = self.arena
        per = -(-a.numel // self.world)
        self.shard = -(-per // ALIGN) * ALIGN
        self.lo = min(self.rank * self.shard, a.numel)
        self.hi = min(self.lo + self.shard, a.numel)
        dev = a.data.device
        # full-size moments from FusedAdam are replaced by this rank's slice
        self.exp_avg = torch.zeros(self.shard, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(self.shard, dtype=torch.float32, device=dev)
        self._gpad = torch.zeros(self.shard * self.world, dtype=torch.float32, device=dev)
        self._gshard = torch.zeros(self.shard, dtype=torch.float32, device=dev)
        self._ppad = torch.zeros(self.shard * self.world, dtype=torch.float32, device=dev)
        self.grad_scale = 1.0 / self.world
        self._native = dist.is_initialized() and dist.get_backend(process_group) == "nccl"
        self._clip_pending: Optional[float] = None
        self._last_norm = torch.zeros((), dtype=torch.float32, device=dev)

    # -- collectives ---------------------------------------------------------------------------
    def _reduce_scatter(self) -> None:
        a = self.arena
        self._gpad[:a.numel].copy_(a.grad)
        if self.world == 1:
            self._gshard.copy_(self._gpad)
        elif self._native:
            dist.reduce_scatter_tensor(self._gshard, self._gpad, group=self.pg)
        else:
            dist.all_reduce(self._gpad, group=self.pg)
            self._gshard.copy_(self._gpad[self.rank * self.shard:(self.rank + 1) * self.shard])

    def _all_gather(self) -> None:
        a = self.arena
        mine = self._ppad[self.rank * self.shard:(self.rank + 1) * self.shard]
        mine.zero_()
        mine[:self.hi - self.lo].copy_(a.data[self.lo:self.hi])
        if self.world > 1:
            if self._native:
                dist.all_gather_into_tensor(self._ppad, mine.clone(), group=self.pg)
            else:
                parts = list(self._ppad.chunk(self.world))
                dist.all_gather(parts, mine.clone(), group=self.pg)
        a.data.copy_(self._ppad[:a.numel])
        if self.shadow is not None:
            self.shadow.copy_(a.data)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self.step_count += 1
        a = self.arena
        if not a.grads_attached():
            a.attach_grads()
        self._reduce_scatter()
        if self.skip_flag is not None:
            # the caller's flag came from this rank's LOCAL (un-reduced) gradient; a non-finite
            # value on any rank lands in some rank's reduced shard, so decide from the shards and
            # agree over the group (MAX) - every rank skips together, no NaN reaches the all-gather
            n = self.hi - self.lo
            bad = torch.zeros(1, dtype=torch.int32, device=self._gshard.device)
            if n > 0:
                # exact per-element test (a shard sum of large finite values could overflow to Inf);
                # the same pbx_nonfinite_flag kernel as the non-ZeRO path on a GPU
                if _hip_ok(self._gshard):
                    from ..ops import _lib
                    ws = torch.empty(1025, dtype=torch.int32, device=self._gshard.device)
                    _lib.call("pbx_nonfinite_flag", self._gshard.data_ptr(), n, ws.data_ptr(), ws[1024:].data_ptr(),
                              float("inf"), 0, _lib.stream_ptr(self._gshard.device))
                    bad = ws[1024:].clone()
                else:
                    bad.fill_(0 if bool(torch.isfinite(self._gshard[:n]).all()) else 1)
            if self.world > 1:
                dist.all_reduce(bad, op=dist.ReduceOp.MAX, group=self.pg)
            self.skip_flag = bad
        if self._clip_pending is not None:
            self._apply_clip()
        n = self.hi - self.lo
        if n > 0:
            p = a.data[self.lo:self.hi]
            g = self._gshard[:n]
            m, v = self.exp_avg[:n], self.exp_avg_sq[:n]
            if _hip_ok(a.data):
                from ..ops import _lib
                self.prepare()
                self._step_dev.add_(1.0)
                sh = self.shadow[self.lo:self.hi] if self.shadow is not None else None
                _lib.call("pbx_adam_flat", p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), _lib.ptr(sh), n,
                          self._hp_dev.data_ptr(), _lib.ptr(self.skip_flag), self._step_dev.data_ptr(),
                          _lib.stream_ptr(a.data.device))
            elif not skip_requested(self.skip_flag):
                adam_update_host(self, p, g, m, v)
        self._all_gather()
        return loss

    @torch.no_grad()
    def clip_grad_norm_(self, max_norm: float) -> torch.Tensor:
        """Deferred global-norm clip: the reduced gradient only exists after ``step()``'s
        reduce-scatter, so the clip is applied there (norm of the mean gradient = sqrt of the
        all-reduced shard sums of squares; same ``max_norm / (norm + 1e-6)`` rule as FusedAdam).
        Returns a 0-dim tensor that ``step()`` fills with the pre-clip norm."""
        self._clip_pending = float(max_norm)
        return self._last_norm

    def _apply_clip(self) -> None:
        n = self.hi - self.lo
        g = self._gshard[:n] * self.grad_scale
        sumsq = (g * g).sum().reshape(1) if n > 0 else self._gshard.new_zeros(1)
        if self.world > 1:
            dist.all_reduce(sumsq, group=self.pg)
        norm = sumsq.sqrt()
        self._last_norm.copy_(norm[0])
        coef = torch.clamp(self._clip_pending / (norm + 1e-6), max=1.0)
        self._gshard.mul_(coef)
        self._clip_pending = None

    # -- checkpoints: gather the full moments so the format is torch.optim.Adam's -------------------
    def _full(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.zeros(self.shard * self.world, dtype=t.dtype, device=t.device)
        if self.world == 1:
            out.copy_(t)
        elif self._native:
            dist.all_gather_into_tensor(out, t.contiguous(), group=self.pg)
        else:
            dist.all_gather(list(out.chunk(self.world)), t.contiguous(), group=self.pg)
        return out[:self.arena.numel]

    def state_dict(self) -> Dict[str, Any]:
        """Collective: every rank of the group must call it."""
        mine = (self.exp_avg, self.exp_avg_sq)
        self.exp_avg, self.exp_avg_sq = self._full(mine[0]), self._full(mine[1])
        try:
            return super().state_dict()
        finally:
            self.exp_avg, self.exp_avg_sq = mine

    @torch.no_grad()
    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        mine = (self.exp_avg, self.exp_avg_sq)
        dev = mine[0].device
        self.exp_avg = torch.zeros(self.arena.numel, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(self.arena.numel, dtype=torch.float32, device=dev)
        try:
            super().load_state_dict(state_dict)
            n = self.hi - self.lo
            mine[0].zero_()
            mine[1].zero_()
            mine[0][:n].copy_(self.exp_avg[self.lo:self.hi])
            mine[1][:n].copy_(self.exp_avg_sq[self.lo:self.hi])
        finally:
            self.exp_avg, self.exp_avg_sq = mine


__all__ = ["ZeroFusedAdam"]
