"""Native threaded pretraining loader over a ``.pbxds`` store (``ops/csrc/pbx_loader.cpp``).

Replaces ``DataLoader(UniRefGO_HDF5PretrainingDataset, shuffle=True, num_workers=N, pin_memory=True)``
(reference ``ProteinBERT/utils.py:96-105``, ``data_processing.py:146-183``):

* C++ worker threads (no Python, no GIL, no worker processes) build *compact clean* batches from
  the memory-mapped store: ``uint8 tokens[B, L]`` (tokenize + reference crop + pad) and the stored
  annotation bit rows ``uint8[B, ceil(A/8)]`` - ~0.4 MB per B=256, L=512 batch;
* the batch is copied from pinned memory to the GPU and expanded + corrupted there by two HIP
  kernels (``pbx_unpack_batch``, ``pbx_corrupt_batch``), giving the reference ``(X, Y, W)`` triple;
* order is a per-epoch seeded permutation of this rank's shard (``rank::world_size``) and the
  stream can resume at any batch (``state_dict``/``load_state_dict``), independent of thread count.

On CPU the same compact batches are expanded with NumPy and corrupted by the torch oracle
(:func:`.synthetic.corrupt_batch_torch`).  Loss weights are float32 here (the reference's float64
weights only promote the loss dtype).
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Iterator, Optional, Tuple

import numpy as np
import torch

from .store import ProteinStore, PbxdsStore
from .synthetic import CorruptionParams, corrupt_batch_torch
from .vocab import create_amino_acid_vocab

Batch = Tuple[Dict[str, torch.Tensor], Dict[str, torch.Tensor], Dict[str, torch.Tensor]]

_P, _I, _I64, _U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64
_bound = False


def _host():
    global _bound
    from ..ops import _lib
    h = _lib.host_lib()
    if not _bound:
        h.pbxl_open.argtypes = [ctypes.c_char_p, _I, _P, ctypes.c_char_p, _I]
        h.pbxl_open.restype = _P
        h.pbxl_size.argtypes = [_P]
        h.pbxl_size.restype = _I64
        h.pbxl_close.argtypes = [_P]
        h.pbxl_close.restype = None
        h.pbxl_loader_create.argtypes = [_P, _I, _I, _P, _I64, _U64, _I, _I, _I, _I, _I, _I64, ctypes.c_char_p, _I]
        h.pbxl_loader_create.restype = _P
        h.pbxl_batches_per_epoch.argtypes = [_P]
        h.pbxl_batches_per_epoch.restype = _I64
        h.pbxl_next.argtypes = [_P, _P, _P, _P]
        h.pbxl_next.restype = _I
        h.pbxl_loader_destroy.argtypes = [_P]
        h.pbxl_loader_destroy.restype = None
        _bound = True
    return h


def native_loader_available() -> bool:
    from ..ops.build import HOST_LIB
    return os.path.exists(HOST_LIB)


class NativeStoreLoader:
    def __init__(self, path: str, batch_size: int, seq_max_length: int, device="cpu", rank: int = 0,
                 world_size: int = 1, shuffle: bool = True, seed: int = 0, drop_last: bool = True,
                 include_last_window: bool = False, num_threads: int = 4, prefetch: int = 8,
                 corruption: CorruptionParams = CorruptionParams(), start_batch: int = 0):
        store = ProteinStore.open(path)
        if not isinstance(store, PbxdsStore):
            raise ValueError("the native loader reads .pbxds stores (convert HDF5 with the ETL CLI)")
        self.path, self.B, self.L = path, int(batch_size), int(seq_max_length)
        self.A = store.n_annotations
        self.nbytes = (self.A + 7) // 8
        self.device = torch.device(device)
        self.rank, self.world_size = rank, world_size
        self.shuffle, self.drop_last, self.include_last_window = shuffle, drop_last, include_last_window
        self.seed = (int(seed) * 1000003 + rank * 7919) & (2**63 - 1)
        self.num_threads, self.prefetch = int(num_threads), int(prefetch)
        self.corruption = corruption
        self.n_total = len(store)
        self.indices = np.arange(rank, self.n_total, world_size, dtype=np.int64)
        if len(self.indices) == 0:
            raise ValueError("empty shard")
        lut = create_amino_acid_vocab().byte_lut.astype(np.uint8)
        self._lut = np.ascontiguousarray(lut)
        err = ctypes.create_string_buffer(512)
        h = _host()
        self._store = h.pbxl_open(path.encode(), self.A, self._lut.ctypes.data, err, 512)
        if not self._store:
            raise RuntimeError(f"pbxl_open: {err.value.decode()}")
        self._loader = None
        self._consumed = int(start_batch)
        self._start(self._consumed)
        # staging: pinned host buffers (ring of 2) + device buffers
        pin = self.device.type == "cuda"
        self._h_tok = [torch.empty((self.B, self.L), dtype=torch.uint8, pin_memory=pin) for _ in range(2)]
        self._h_bits = [torch.empty((self.B, self.nbytes), dtype=torch.uint8, pin_memory=pin) for _ in range(2)]
        self._events = [None, None]
        self._slot = 0
        self._bid = ctypes.c_int64(0)
        if pin:
            self._d_tok = torch.empty((self.B, self.L), dtype=torch.uint8, device=self.device)
            self._d_bits = torch.empty((self.B, self.nbytes), dtype=torch.uint8, device=self.device)
        self._gen = torch.Generator(device=self.device)
        self._gen.manual_seed(self.seed)

    # ------------------------------------------------------------------------------------------
    def _start(self, start_batch: int) -> None:
        err = ctypes.create_string_buffer(512)
        self._loader = _host().pbxl_loader_create(
            self._store, self.B, self.L, self.indices.ctypes.data, len(self.indices), self.seed, int(self.shuffle),
            int(self.drop_last), int(self.include_last_window), self.num_threads, self.prefetch, int(start_batch),
            err, 512)
        if not self._loader:
            raise RuntimeError(f"pbxl_loader_create: {err.value.decode()}")
        self.batches_per_epoch = int(_host().pbxl_batches_per_epoch(self._loader))

    def __len__(self) -> int:
        return self.batches_per_epoch

    @property
    def epoch(self) -> int:
        return self._consumed // self.batches_per_epoch

    def state_dict(self) -> Dict[str, int]:
        return {"batch": self._consumed, "seed": self.seed, "world_size": self.world_size, "rank": self.rank}

    def load_state_dict(self, st: Dict[str, int]) -> None:
        if st.get("world_size", self.world_size) != self.world_size:
            raise ValueError("loader state was saved with a different world size")
        _host().pbxl_loader_destroy(self._loader)
        self._consumed = int(st["batch"])
        self._start(self._consumed)

    def close(self) -> None:
        h = _host()
        if self._loader:
            h.pbxl_loader_destroy(self._loader)
            self._loader = None
        if self._store:
            h.pbxl_close(self._store)
            self._store = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    # ------------------------------------------------------------------------------------------
    def next_clean_compact(self) -> Tuple[torch.Tensor, torch.Tensor, int]:
        """Next compact batch into a pinned staging slot: (tokens u8 [B,L], bits u8 [B,nbytes], rows)."""
        s = self._slot
        self._slot ^= 1
        if self._events[s] is not None:
            self._events[s].synchronize()       # the H2D copy that last read this slot is done
        rows = _host().pbxl_next(self._loader, self._h_tok[s].data_ptr(), self._h_bits[s].data_ptr(),
                                 ctypes.byref(self._bid))
        if rows < 0:
            raise RuntimeError("native loader stopped")
        self._consumed += 1
        return self._h_tok[s], self._h_bits[s], rows, s

    def next_batch(self) -> Batch:
        tok_h, bits_h, rows, s = self.next_clean_compact()
        if self.device.type == "cuda":
            from ..ops import corrupt as corrupt_op
            self._d_tok.copy_(tok_h, non_blocking=True)
            self._d_bits.copy_(bits_h, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._events[s] = ev
            tokens, ann = corrupt_op.unpack_batch(self._d_tok, self._d_bits, self.A)
            out = corrupt_op.corrupt_batch(tokens, ann, self.corruption, seed=self.seed, step=self._consumed)
        else:
            tokens = tok_h.long()
            bits = np.unpackbits(bits_h.numpy(), axis=1, bitorder="little")[:, :self.A]
            ann = torch.from_numpy(bits.astype(np.float32))
            out = corrupt_batch_torch(tokens, ann, self.corruption, self._gen, weights_dtype=torch.float32)
        if rows < self.B:   # last partial batch (drop_last=False)
            out = tuple({k: v[:rows] for k, v in d.items()} for d in out)
        return out

    def __iter__(self) -> Iterator[Batch]:
        """One epoch (the remainder of the current one when resumed mid-epoch)."""
        left = self.batches_per_epoch - (self._consumed % self.batches_per_epoch)
        for _ in range(left):
            yield self.next_batch()
