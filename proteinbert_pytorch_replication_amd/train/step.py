"""One pretraining step: loss -> backward (+ overlapped DP all-reduce) -> fused Adam.

Reference step body: ``ProteinBERT/utils.py:287-301`` (H2D copies, forward,
weighted CE + BCE, ``.item()`` sync, zero_grad / backward / step).  Here the
step never synchronises with the host: the loss stays on the device, the
non-finite check is a device flag consumed by the fused Adam kernel, and on
a GPU the forward/backward run through the fused HIP kernels
(:mod:`..ops.fused_model`) with bf16 activations.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from .losses import pretrain_loss_torch, is_standard_loss_pair
from .optim import FusedAdam


def resolve_compute_dtype(spec, device: torch.device) -> torch.dtype:
    if isinstance(spec, torch.dtype):
        return spec
    if spec in (None, "auto"):
        return torch.bfloat16 if device.type == "cuda" else torch.float32
    return {"bf16": torch.bfloat16, "fp32": torch.float32, "float32": torch.float32,
            "bfloat16": torch.bfloat16}[spec]


class PretrainStep:
    def __init__(self, model, optimizer, ddp=None, local_loss_fn=None, global_loss_fn=None,
                 compute_dtype="auto", grad_clip: Optional[float] = None, skip_nonfinite: bool = True):
        self.model = model
        self.optimizer = optimizer
        self.ddp = ddp
        self.local_loss_fn = local_loss_fn
        self.global_loss_fn = global_loss_fn
        self.standard_loss = is_standard_loss_pair(local_loss_fn, global_loss_fn)
        self.device = next(model.parameters()).device
        self.compute_dtype = resolve_compute_dtype(compute_dtype, self.device)
        self.grad_clip = grad_clip
        self.skip_nonfinite = skip_nonfinite
        self.fused = isinstance(optimizer, FusedAdam)
        self.last_parts = None
        if self.fused and ddp is not None and ddp.enabled:
            optimizer.grad_scale = 1.0 / ddp.world

    def loss(self, X: Dict[str, torch.Tensor], Y: Dict[str, torch.Tensor], W: Dict[str, torch.Tensor],
             return_parts: bool = False):
        m = self.model
        if m.resolved_backend(self.device) == "hip" and self.standard_loss:
            from ..ops.fused_model import fused_pretrain_loss
            return fused_pretrain_loss(m, X, Y, W, return_parts=return_parts)
        h, g = m.encode_torch(X["local"], X["global"], compute_dtype=self.compute_dtype)
        pl, pg = m.heads_torch(h, g)
        return pretrain_loss_torch(pl, pg, Y, {k: v.float() for k, v in W.items()}, m.semantics,
                                   None if self.standard_loss else self.local_loss_fn,
                                   None if self.standard_loss else self.global_loss_fn, return_parts)

    def overlapped_optimizer(self) -> bool:
        """DP with the fused Adam and no gradient clipping (which needs the global norm first): the
        update of every gradient bucket but the last runs beside the last bucket's all-reduce
        (:meth:`..parallel.ddp.BucketedAllReduce.finish_and_step`)."""
        return (self.ddp is not None and self.ddp.enabled and type(self.optimizer) is FusedAdam
                and self.grad_clip is None and getattr(self.ddp, "overlap_optimizer", True))

    def __call__(self, X, Y, W) -> torch.Tensor:
        opt = self.optimizer
        opt.zero_grad()
        overlap = self.overlapped_optimizer()
        if overlap:
            self.ddp.begin_overlapped_step()
        loss, l_local, l_global = self.loss(X, Y, W, return_parts=True)
        # device scalars (no host sync): the per-head losses of the last step, for the metrics
        self.last_parts = (l_local.detach(), l_global.detach())
        if self.model.resolved_backend(self.device) == "hip":
            from ..ops.global_track import unit_loss_grad, unit_seed
            from ..ops import streams
            with unit_loss_grad():
                torch.autograd.backward(loss, unit_seed(loss))
            streams.join()                      # conv weight gradients ran on the aux stream
        else:
            loss.backward()
        if overlap:
            self.ddp.finish_and_step(opt, self.skip_nonfinite)
            return loss.detach()
        if self.ddp is not None:
            self.ddp.finish(average=not self.fused)
        if self.grad_clip is not None:
            if self.fused:
                opt.clip_grad_norm_(self.grad_clip)
            else:
                torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.grad_clip)
        if self.fused and self.skip_nonfinite:
            # all-reduced grads (bucketed DP): every rank takes the same decision, no host sync.
            # ZeroFusedAdam reduces inside step() and replaces this local flag by a group-wide
            # decision over the reduced shards (parallel/zero.py)
            opt.set_nonfinite_skip()
        opt.step()
        return loss.detach()


class PrefetchedBatches:
    """Device-side batch producer run one step ahead on its own HIP stream.

    ``batch_fn()`` enqueues the generation of a batch (synthetic data + corruption kernels, or an H2D
    copy) on the current stream.  Here batch i + 1 is enqueued on a side stream when batch i is handed
    out, so its small, latency-bound kernels run beside the training step instead of at the head of
    the next one; the consumer stream waits on an event recorded after the batch (the reference's
    loader hands the step a ready batch the same way, ``utils.py:282-289``).  Every batch is still
    produced inside the consumer's loop; the extra one is only ever the next step's."""

    def __init__(self, batch_fn, device: torch.device):
        self.batch_fn = batch_fn
        self.device = device
        self.stream = torch.cuda.Stream(device=device)
        self._next = None

    def _make(self):
        if self._next is None:
            # once: the producer's device state (RNG / step counters) was created on the consumer stream
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            batch = self.batch_fn()
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return batch, ev

    def __call__(self):
        if self._next is None:
            self._next = self._make()
        batch, ev = self._next
        main = torch.cuda.current_stream(self.device)
        main.wait_event(ev)
        for part in batch:
            for t in (part.values() if isinstance(part, dict) else (part,)):
                if isinstance(t, torch.Tensor):
                    t.record_stream(main)       # allocated on the side stream, consumed on this one
        self._next = self._make()
        return batch


class GraphedStep:
    """The whole training step captured once as a hipGraph and replayed.

    Captures data generation (when ``batch_fn`` produces the batch on the device), forward, the fused
    loss, backward, the (optional) DP all-reduce and the fused Adam update: ~290 kernel launches
    become one ``hipGraphLaunch``, so the host never throttles the GPU.  Everything the replay reads
    that changes between steps lives in device memory (synthetic-data and Adam step counters, Adam
    hyper-parameters refreshed by :meth:`FusedAdam.prepare` before each replay).
    """

    def __init__(self, step: PretrainStep, batch_fn, warmup: int = 2):
        if not torch.cuda.is_available():
            raise RuntimeError("GraphedStep needs a GPU")
        self.step = step
        self.batch_fn = batch_fn
        opt = step.optimizer
        if not isinstance(opt, FusedAdam):
            raise TypeError("GraphedStep needs the FusedAdam optimizer (device-side hyper-parameters)")
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                X, Y, W = batch_fn()
                step(X, Y, W)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        opt.prepare()
        self.graph = torch.cuda.CUDAGraph()
        # with a process group attached, the RCCL watchdog thread polls its work events while this thread
        # captures: under the default "global" mode such a call from another thread invalidates the capture
        # (seen as a rare hipErrorStreamCaptureInvalidated in the DP capture test), so only this thread's
        # calls are checked
        ddp = getattr(step, "ddp", None)
        mode = "thread_local" if ddp is not None and getattr(ddp, "enabled", False) else "global"
        with torch.cuda.graph(self.graph, capture_error_mode=mode):
            X, Y, W = batch_fn()
            self.loss = step(X, Y, W)
        # capture recorded the optimizer step without executing it: undo the host-side increment
        opt.step_count -= 1

    def __call__(self) -> torch.Tensor:
        opt = self.step.optimizer
        opt.step_count += 1
        opt.prepare()
        self.graph.replay()
        return self.loss
