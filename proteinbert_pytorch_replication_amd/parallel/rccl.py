"""Direct RCCL communicator for the gradient buckets.

``torch.distributed.all_reduce`` on the ``nccl`` backend runs every collective on ProcessGroupNCCL's own
internal stream: the call records an event on the caller's stream, makes the internal stream wait for it,
and ``work.wait()`` makes the caller wait back.  HIP multiplexes streams onto ``GPU_MAX_HW_QUEUES``
hardware queues (4 on the MI355X pool) and a cross-stream wait is a barrier packet that holds its whole
hardware queue: the training step already keeps four streams busy (the main stream, the conv
weight-gradient stream and the two head / input-layer streams), so the process group's stream is a fifth
that shares a hardware queue with one of them, and each bucket's wait for the weight-gradient stream
stalls whatever shares it (a forced 1-rank RCCL step ran +3.7 ms over the eager step,
``profiles/r5/dp_host_and_flags.txt``; no RCCL kernel of that step took measurable time,
``profiles/r6/dp_trace_before.txt``).

This module keeps a second RCCL communicator over the same ranks, created through RCCL's C API (the
library torch itself loaded, so one RCCL instance per process), and enqueues ``ncclAllReduce`` directly
on the stream the caller names -- the weight-gradient stream that produces each bucket's last gradients
(``ops/streams.py``).  No extra stream, no event pair per collective, and the calls are hipGraph-capturable
like any other launch on that stream.  The unique id travels through the process group's rendezvous store.

Only the gradient buckets and the 4-byte non-finite flag use it (``parallel/ddp.py``); everything else
(parameter broadcast, loss reductions, barriers) stays on the process group.  ``PBX_DP_COMM=torch`` keeps
the process-group path.
"""
from __future__ import annotations

import ctypes
import itertools
import os
import threading
from typing import Optional

import torch
import torch.distributed as dist

NCCL_UNIQUE_ID_BYTES = 128
# ncclDataType_t / ncclRedOp_t values (rccl.h)
_DTYPES = {torch.float32: 7, torch.bfloat16: 9, torch.float16: 6, torch.int32: 2, torch.int64: 4,
           torch.float64: 8}
_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3}


class _UniqueId(ctypes.Structure):
    # c_ubyte, not c_char: a c_char array field reads back as a NUL-terminated string (truncated at the
    # first zero byte of the id)
    _fields_ = [("internal", ctypes.c_ubyte * NCCL_UNIQUE_ID_BYTES)]


class RcclError(RuntimeError):
    pass


_lib_handle: Optional[ctypes.CDLL] = None
_lock = threading.Lock()
_serial = itertools.count()


def library_path() -> str:
    """The librccl torch was built against (already mapped into this process by libtorch_hip)."""
    tl = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    if os.path.exists(tl):
        return tl
    for p in ("/opt/rocm/lib/librccl.so", "/opt/rocm/lib/librccl.so.1"):
        if os.path.exists(p):
            return p
    raise RcclError("librccl.so not found")


def _rccl() -> ctypes.CDLL:
    global _lib_handle
    with _lock:
        if _lib_handle is None:
            lib = ctypes.CDLL(library_path(), mode=ctypes.RTLD_GLOBAL)
            lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
            lib.ncclGetUniqueId.restype = ctypes.c_int
            lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _UniqueId, ctypes.c_int]
            lib.ncclCommInitRank.restype = ctypes.c_int
            lib.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
            lib.ncclAllReduce.restype = ctypes.c_int
            lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
            lib.ncclCommDestroy.restype = ctypes.c_int
            lib.ncclGetErrorString.argtypes = [ctypes.c_int]
            lib.ncclGetErrorString.restype = ctypes.c_char_p
            _lib_handle = lib
    return _lib_handle


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = _rccl().ncclGetErrorString(rc)
        raise RcclError(f"{what}: RCCL error {rc} ({msg.decode() if msg else '?'})")


def _store():
    from torch.distributed import distributed_c10d as c10d
    return c10d._get_default_store()


def exchange_unique_id(rank: int, key: str, make_id) -> bytes:
    """Rank 0 creates the id (``make_id() -> bytes``) and publishes it under ``key`` in the process
    group's store; every rank returns it.  Pure store traffic (tested on gloo without a GPU)."""
    st = _store()
    if rank == 0:
        uid = make_id()
        st.set(key, uid)
        return uid
    st.wait([key])
    return st.get(key)


class Communicator:
    """One RCCL communicator over the ranks of ``group`` (the default group when None)."""

    def __init__(self, group=None, device: Optional[torch.device] = None):
        if not dist.is_initialized():
            raise RcclError("torch.distributed is not initialised")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        lib = _rccl()
        ranks = dist.get_process_group_ranks(group) if group is not None else list(range(self.world))
        key = f"pbx_rccl_uid/{'-'.join(map(str, ranks))}/{next(_serial)}"

        def make_id() -> bytes:
            uid = _UniqueId()
            _check(lib.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
            return bytes(uid.internal)

        raw = exchange_unique_id(self.rank, key, make_id)
        if len(raw) != NCCL_UNIQUE_ID_BYTES:
            raise RcclError(f"unique id of {len(raw)} bytes")
        uid = _UniqueId()
        ctypes.memmove(ctypes.addressof(uid), raw, NCCL_UNIQUE_ID_BYTES)
        comm = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _check(lib.ncclCommInitRank(ctypes.byref(comm), self.world, uid, self.rank), "ncclCommInitRank")
        self._comm = comm
        self._lib = lib

    def all_reduce_(self, t: torch.Tensor, op: str = "sum", stream: Optional[int] = None) -> None:
        """In-place all-reduce of contiguous ``t`` enqueued on ``stream`` (a raw hipStream_t; the current
        stream when None).  Stream-ordered: nothing to wait for on the host."""
        if self._comm is None:
            raise RcclError("communicator destroyed")
        if not (t.is_cuda and t.is_contiguous()):
            raise ValueError("all_reduce_: a contiguous device tensor is required")
        dt = _DTYPES.get(t.dtype)
        if dt is None:
            raise ValueError(f"all_reduce_: dtype {t.dtype}")
        if stream is None:
            from ..ops import _lib as _pbx
            stream = _pbx.stream_ptr(t.device)
        _check(self._lib.ncclAllReduce(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(t.data_ptr()),
                                       ctypes.c_size_t(t.numel()), dt, _OPS[op], self._comm,
                                       ctypes.c_void_p(stream)), "ncclAllReduce")

    def close(self) -> None:
        if self._comm is not None:
            torch.cuda.synchronize(self.device)
            self._lib.ncclCommDestroy(self._comm)
            self._comm = None


def wanted(group=None) -> bool:
    """Use a direct communicator for this group: the nccl (RCCL) backend on a GPU, unless
    ``PBX_DP_COMM=torch``."""
    if os.environ.get("PBX_DP_COMM", "rccl") != "rccl":
        return False
    if not (dist.is_initialized() and torch.cuda.is_available()):
        return False
    return dist.get_backend(group) == "nccl"
