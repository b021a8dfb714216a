"""Data-parallel batch-axis softmax of the reference local head (``dp_batch_softmax``).

The reference's local output is ``nn.Softmax()`` with the implicit dim, which for the ``[B, L, V]`` logits
is the BATCH axis (``ProteinBERT/modules.py:277-284``): every (position, token) is
normalised over the samples of the batch.  Plain data parallelism therefore changes the model -- each
rank normalises over its own micro-batch.  With this option enabled the ranks of a process group share
the batch axis, so DP=N with micro-batch b computes exactly the single-process batch-N·b step:

    forward   M[l,v] = max over ALL ranks' samples of z      (all-reduce MAX,  [L, V] floats)
              S[l,v] = sum over ALL samples of exp(z - M)     (all-reduce SUM,  [L, V] floats)
    backward  T[l,v] = sum over ALL samples of p * g          (all-reduce SUM,  [L, V] floats)
              dz     = p (g - T)

Each rank keeps its own loss mean over its b·L rows and the DP gradient average divides by the world
size, which together give the gradient of the global-batch mean (``ProteinBERT/utils.py:293``).  The
fused HIP head (``csrc/lhead.hip`` stages A/B/C) runs the same three reductions between its passes; the
PyTorch path uses :class:`DPBatchSoftmax`.

Off by default: the three reductions are small (``[L, 32]`` float2 each) but sit on the forward critical
path, and the single-launch head (B <= 1024) is replaced by the five-pass form.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

_STATE = {"on": False, "group": None, "force": False}


def enable(group=None, force: bool = False) -> None:
    """Share the local head's batch-axis softmax over the ranks of ``group`` (default: the world).
    ``force``: run the shared form even on a 1-rank group (its cost on one GPU, tools/cpu_overhead.py)."""
    if not dist.is_initialized():
        raise RuntimeError("dp_batch_softmax needs an initialised process group")
    _STATE.update(on=True, group=group, force=force)


def disable() -> None:
    _STATE.update(on=False, group=None, force=False)


def active() -> bool:
    """True when enabled over more than one rank (a 1-rank group is the plain softmax unless forced)."""
    return _STATE["on"] and dist.is_initialized() and (_STATE["force"] or dist.get_world_size(_STATE["group"]) > 1)


def all_reduce_(t: torch.Tensor, op: str) -> torch.Tensor:
    """In-place all-reduce in stream order (``op``: "sum" | "max")."""
    rop = dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX
    group = _STATE["group"]
    if t.is_cuda and dist.get_backend(group) == "gloo":
        # gloo's CUDA collectives are not ordered with the caller's stream on every build: stage on the host
        h = t.cpu()
        dist.all_reduce(h, op=rop, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=rop, group=group)
    return t


def merge_max_sum(m: torch.Tensor, s: torch.Tensor) -> tuple:
    """Per-rank (max, sum exp(z - max)) -> the group's (M, S), same shapes (new tensors)."""
    mg = all_reduce_(m.clone(), "max")
    sg = all_reduce_(s * torch.exp(m - mg), "sum")
    return mg, sg


def merge_head_stats(ms: torch.Tensor) -> None:
    """The fused head's raw (M, S) image ``[L, 32, 2]`` (stage A, raw) -> the group's (M, 1/S), in place."""
    mg, sg = merge_max_sum(ms[..., 0].contiguous(), ms[..., 1].contiguous())
    ms[..., 0] = mg
    ms[..., 1] = torch.where(sg > 0, 1.0 / sg.clamp_min(torch.finfo(torch.float32).tiny), torch.zeros_like(sg))


class DPBatchSoftmax(torch.autograd.Function):
    """softmax over dim 0 of ``z [b, ...]`` with the batch axis spanning every rank of the group."""

    @staticmethod
    def forward(ctx, z: torch.Tensor) -> torch.Tensor:
        zf = z.float()
        m, _ = zf.max(dim=0)
        e = torch.exp(zf - m)
        mg, sg = merge_max_sum(m, e.sum(dim=0))
        p = torch.exp(zf - mg) / sg
        ctx.save_for_backward(p)
        return p.to(z.dtype)

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        (p,) = ctx.saved_tensors
        gf = g.float()
        t = all_reduce_((p * gf).sum(dim=0), "sum")
        return (p * (gf - t)).to(g.dtype)


def softmax_over_batch(z: torch.Tensor) -> torch.Tensor:
    """The reference local head's softmax: over this rank's batch, or the DP group's when enabled."""
    if active():
        return DPBatchSoftmax.apply(z)
    return torch.softmax(z, dim=0)


def group() -> Optional[object]:
    return _STATE["group"]
