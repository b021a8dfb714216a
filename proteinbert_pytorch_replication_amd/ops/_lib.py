"""ctypes binding of the in-tree HIP library (``libpbx_hip.so``).

The library must be loaded *after* ``import torch`` so that it binds to the
HIP runtime torch already loaded (same ``libamdhip64.so.7`` soname).  Every
launcher returns a ``hipError_t``; a non-zero code raises.  On a GPU box a
missing library is an error, never a silent fallback to eager ops.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

from .build import HIP_LIB as _BUILT_HIP_LIB, HIP_LIB_EXACT as _BUILT_HIP_LIB_EXACT, HOST_LIB

GELU_MODES = ("fitted", "exact")


def _default_lib() -> str:
    mode = os.environ.get("PBX_GELU", "fitted")
    if mode not in GELU_MODES:
        raise ValueError(f"PBX_GELU={mode!r}: expected one of {GELU_MODES}")
    return _BUILT_HIP_LIB_EXACT if mode == "exact" else _BUILT_HIP_LIB


# The GELU core of the fused kernels: "fitted" (libpbx_hip.so, the default) or "exact" (libpbx_hip_exact.so,
# the erf form of the reference's nn.GELU()), chosen by PBX_GELU / set_gelu() before the first kernel launch.
# PBX_HIP_LIB: load any other build of the kernel library (A/B comparisons of kernel variants).
HIP_LIB = os.environ.get("PBX_HIP_LIB") or _default_lib()


def gelu_mode() -> str:
    return "exact" if HIP_LIB == _BUILT_HIP_LIB_EXACT else ("fitted" if HIP_LIB == _BUILT_HIP_LIB else "custom")


def set_gelu(mode: str) -> None:
    """Select the fused kernels' GELU core ("fitted" | "exact") for this process.  Must precede the first
    kernel launch (the library is loaded once); a later call with another mode raises."""
    global HIP_LIB
    if mode not in GELU_MODES:
        raise ValueError(f"gelu mode {mode!r}: expected one of {GELU_MODES}")
    want = _BUILT_HIP_LIB_EXACT if mode == "exact" else _BUILT_HIP_LIB
    if want == HIP_LIB:
        return
    if _lib is not None:
        raise HipError(f"set_gelu({mode!r}): the kernel library ({HIP_LIB}) is already loaded")
    HIP_LIB = want
    os.environ["PBX_GELU"] = mode     # child processes (DP ranks spawned later) inherit the choice

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int
_F32 = ctypes.c_float

# name -> argtypes (all return int hipError_t)
_SIGS = {
    "pbx_adam_flat": [_P, _P, _P, _P, _P, _I64, _P, _P, _P, _P],
    "pbx_sumsq_flat": [_P, _I64, _P, _P, _P],
    "pbx_clip_scale_flat": [_P, _I64, _P, _F32, _P],
    "pbx_nonfinite_flag": [_P, _I64, _P, _P, _F32, _I32, _P],
    "pbx_fill_flat": [_P, _I64, _F32, _P],
    "pbx_add_scalar": [_P, _F32, _P],
    "pbx_add_i64": [_P, _I64, _P],
    "pbx_colsum_set": [_P, _I32, _I32, _P, _P, _P],
}

_lib: Optional[ctypes.CDLL] = None
_host: Optional[ctypes.CDLL] = None


class HipError(RuntimeError):
    pass


def available() -> bool:
    return os.path.exists(HIP_LIB)


def register(name: str, argtypes) -> None:
    """Kernel modules declare their launchers here (before first use)."""
    _SIGS[name] = argtypes
    if _lib is not None:
        fn = getattr(_lib, name, None)
        if fn is not None:
            fn.argtypes, fn.restype = argtypes, ctypes.c_int


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(HIP_LIB):
            raise HipError(f"HIP kernel library not built: {HIP_LIB}. "
                           f"Run `python -m proteinbert_pytorch_replication_amd.ops.build`.")
        _ = torch.cuda.is_available()  # make sure torch's HIP runtime is loaded first
        _lib = ctypes.CDLL(HIP_LIB, mode=ctypes.RTLD_LOCAL)
        for name, args in _SIGS.items():
            fn = getattr(_lib, name, None)
            if fn is None:       # an older A/B build (PBX_HIP_LIB) without this launcher: call() raises
                continue
            fn.argtypes, fn.restype = args, ctypes.c_int
    return _lib


def host_lib() -> ctypes.CDLL:
    global _host
    if _host is None:
        if not os.path.exists(HOST_LIB):
            raise HipError(f"host library not built: {HOST_LIB}")
        _host = ctypes.CDLL(HOST_LIB, mode=ctypes.RTLD_LOCAL)
    return _host


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device: Optional[torch.device] = None) -> int:
    """Raw hipStream_t of the current stream (the step issues ~200 launches: the torch.cuda.Stream
    wrapper object per launch cost ~8 us of host time each)."""
    if _raw_stream is not None:
        idx = device.index if device is not None and device.index is not None else torch.cuda.current_device()
        return _raw_stream(idx)
    return torch.cuda.current_stream(device).cuda_stream


_FN = {}


def call(name: str, *args) -> None:
    fn = _FN.get(name)
    if fn is None:
        if name not in _SIGS:   # ctypes would pass Python ints as 32-bit C ints and truncate device pointers
            raise HipError(f"{name}: launcher not registered (import the ops module that declares it)")
        fn = getattr(lib(), name, None)
        if fn is None:
            raise HipError(f"{name}: not exported by {HIP_LIB}")
        _FN[name] = fn
    rc = fn(*args)
    if rc != 0:
        raise HipError(f"{name} failed with hipError {rc}")


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()
