"""Process-group bootstrap: one process per GPU, RCCL over xGMI.

The reference has no distributed code at all.  This module
reads the ``torchrun`` environment (``RANK``, ``WORLD_SIZE``,
``LOCAL_RANK``, ``MASTER_ADDR``/``MASTER_PORT``), pins the process to
``cuda:LOCAL_RANK`` and opens a ``"nccl"`` process group — which *is* RCCL on
ROCm.  ``gloo`` is used only when no GPU is present (CPU unit tests).
``HSA_ENABLE_IPC_MODE_LEGACY=0`` is kept (dmabuf IPC is the only mode the
host driver supports).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"
    rccl_env: Optional[dict] = None       # the RCCL settings rccl_node_defaults applied (None: none)

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


_INFO: Optional[DistInfo] = None


def env_world() -> DistInfo:
    return DistInfo(rank=int(os.environ.get("RANK", 0)), world_size=int(os.environ.get("WORLD_SIZE", 1)),
                    local_rank=int(os.environ.get("LOCAL_RANK", 0)))


def _gpu_node_present() -> bool:
    return os.path.exists("/dev/kfd") and os.environ.get("HIP_VISIBLE_DEVICES", "x") != ""


def init_distributed(backend: str = "auto", timeout_s: int = 600, device: Optional[str] = None) -> DistInfo:
    """Idempotent.  With WORLD_SIZE==1 no process group is created."""
    global _INFO
    if _INFO is not None:
        return _INFO
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    info = env_world()
    # the node defaults go into the environment BEFORE the first GPU call: the HSA runtime reads its HSA_*
    # variables once, at start-up.  Decided from the arguments and the environment only: a device query
    # (torch.cuda.device_count() goes through hipGetDeviceCount on builds without amdsmi) could start HSA
    # first; /dev/kfd is the ROCm compute device node
    rccl_env = None
    if info.world_size > 1 and device != "cpu" and backend in ("auto", "nccl") and _gpu_node_present():
        rccl_env = rccl_node_defaults(info.world_size)
    use_gpu = torch.cuda.is_available() and device != "cpu"
    if use_gpu:
        torch.cuda.set_device(info.local_rank)
        info.device = torch.device("cuda", info.local_rank)
    else:
        info.device = torch.device("cpu")
    if info.world_size > 1:
        if backend == "auto":
            backend = "nccl" if use_gpu else "gloo"
        if backend == "nccl":
            info.rccl_env = rccl_env
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = info.device
            opts = nccl_pg_options()
            if opts is not None:
                kw["pg_options"] = opts
        if not dist.is_initialized():
            dist.init_process_group(**kw)
        info.backend = backend
    _INFO = info
    return info


# RCCL defaults for one 8 x MI355X node.  The node's xGMI is a fully connected K8: 7 point-to-
# point links of ~153 GB/s per GPU.  One ring all-reduce is bound by ONE link per direction (2 (7/8) 67 MB /
# 153 GB/s = 0.77 ms for the 67 MB gradient payload); K8 decomposes into 3 edge-disjoint Hamiltonian
# cycles + a perfect matching, i.e. up to 6 link-disjoint directed rings, so the all-reduce needs >= 6
# channels, with a margin for RCCL's per-channel protocol overhead.  These are DEFAULTS: every variable the
# launch environment already sets wins, and PBX_RCCL_DEFAULTS=0 applies none.
RCCL_NODE_DEFAULTS = {
    "NCCL_MIN_NCHANNELS": "16",        # >= 6 directed rings over the K8 links (RCCL may still use more)
    "HSA_NO_SCRATCH_RECLAIM": "1",     # keep RCCL kernels' scratch resident (no reclaim stalls per call)
    "TORCH_NCCL_ASYNC_ERROR_HANDLING": "1",   # a failed / hung collective aborts the job (watchdog)
}


def rccl_node_defaults(world_size: int) -> Optional[dict]:
    """Apply :data:`RCCL_NODE_DEFAULTS` for a single-node multi-GPU job (one process per GPU); returns
    what was set.  Multi-node jobs (LOCAL_WORLD_SIZE < WORLD_SIZE) keep RCCL's own topology tuning."""
    if os.environ.get("PBX_RCCL_DEFAULTS", "1") == "0" or world_size < 2:
        return None
    if int(os.environ.get("LOCAL_WORLD_SIZE", world_size)) != world_size:
        return None
    applied = {}
    # torch.cuda.is_initialized() is False after a bare device query that already started HSA, so this
    # guard is a lower bound: callers set the environment before any HIP call (init_distributed does)
    hsa_started = torch.cuda.is_initialized()
    for k, v in RCCL_NODE_DEFAULTS.items():
        if k.startswith("HSA_") and hsa_started:
            continue                    # read only at HSA start-up: setting it now would change nothing
        if k not in os.environ:
            os.environ[k] = v
            applied[k] = v
    return applied


def nccl_pg_options():
    """RCCL's own streams at high priority: the gradient all-reduce kernels are dispatched ahead of
    the backward kernels they overlap.  ``PBX_RCCL_HIGH_PRIO=0`` turns it off."""
    if os.environ.get("PBX_RCCL_HIGH_PRIO", "1") != "1" or not hasattr(dist, "ProcessGroupNCCL"):
        return None
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    return opts


def get_info() -> DistInfo:
    return _INFO if _INFO is not None else env_world()


def is_main() -> bool:
    return get_info().rank == 0


def barrier() -> None:
    if dist.is_available() and dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_max(x: float, device: Optional[torch.device] = None) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device or get_info().device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_mean_(t: torch.Tensor) -> torch.Tensor:
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t)
        t /= dist.get_world_size()
    return t


def broadcast_module(module: torch.nn.Module, src: int = 0) -> None:
    """Make every rank start from rank 0's parameters and buffers (incl. attention heads)."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src)
    from ..train.arena import invalidate_bf16_mirrors
    invalidate_bf16_mirrors(module.parameters())


def destroy() -> None:
    global _INFO
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _INFO = None
