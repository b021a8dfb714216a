"""On-disk pretraining dataset store (the E3 layout).

The reference writes HDF5 with root-level datasets
(``ProteinBERT/uniref_dataset.py:236-245``)::

    included_annotations[n_ann] str, uniprot_ids[n] str, seqs[n] str,
    seq_lengths[n] int32, annotation_masks[n, n_ann] bool

Two interchangeable backends exist:

* ``.h5``     - the exact reference layout.  Read and written by h5py when it is importable,
  otherwise by the dependency-free implementation in :mod:`.hdf5` (h5py and libhdf5 are not in
  this image);
* ``.pbxds``  - a directory of memory-mappable ``.npy`` arrays with the same
  fields (sequence bytes + offsets, bit-packed annotation masks).  It is what
  the native batch builder (``ops/csrc/pbx_loader.cpp``) reads without
  Python in the loop.

Both expose the same :class:`ProteinStore` reader API.
"""
from __future__ import annotations

import json
import os
from typing import Iterable, List, Optional, Sequence

import numpy as np

try:  # pragma: no cover - h5py is absent in the build image
    import h5py  # type: ignore
except Exception:  # noqa: BLE001
    h5py = None

from . import hdf5 as pbx_h5

PBXDS_VERSION = 1


def has_h5py() -> bool:
    return h5py is not None


def _text(v) -> str:
    return v.decode("utf-8") if isinstance(v, (bytes, np.bytes_)) else str(v)


class ProteinStore:
    """Random-access reader. Use :meth:`open`."""

    @staticmethod
    def open(path: str) -> "ProteinStore":
        if os.path.isdir(path) and os.path.exists(os.path.join(path, "meta.json")):
            return PbxdsStore(path)
        if path.endswith((".h5", ".hdf5")) and os.path.isfile(path):
            return H5Store(path)
        raise FileNotFoundError(f"no dataset store at {path}")

    # interface
    def __len__(self) -> int: ...
    def seq(self, i: int) -> str: ...
    def annotation_mask(self, i: int) -> np.ndarray: ...
    def uniprot_id(self, i: int) -> str: ...
    included_annotations: List[str]


class PbxdsStore(ProteinStore):
    def __init__(self, path: str):
        self.path = path
        with open(os.path.join(path, "meta.json")) as f:
            self.meta = json.load(f)
        if self.meta.get("version") != PBXDS_VERSION:
            raise ValueError(f"unsupported .pbxds version {self.meta.get('version')}")
        ld = lambda name: np.load(os.path.join(path, name), mmap_mode="r", allow_pickle=False)  # noqa: E731
        self.seq_offsets = ld("seq_offsets.npy")
        self.seq_bytes = ld("seq_bytes.npy")
        self.seq_lengths = ld("seq_lengths.npy")
        self.annotation_bits = ld("annotation_bits.npy")
        self.id_offsets = ld("id_offsets.npy")
        self.id_bytes = ld("id_bytes.npy")
        self.n_annotations = int(self.meta["n_annotations"])
        self.included_annotations = list(self.meta["included_annotations"])

    def __len__(self) -> int:
        return int(self.meta["n"])

    def seq(self, i: int) -> str:
        a, b = int(self.seq_offsets[i]), int(self.seq_offsets[i + 1])
        return bytes(self.seq_bytes[a:b]).decode("ascii")

    def annotation_mask(self, i: int) -> np.ndarray:
        bits = np.unpackbits(np.asarray(self.annotation_bits[i]), bitorder="little")
        return bits[:self.n_annotations].astype(bool)

    def uniprot_id(self, i: int) -> str:
        a, b = int(self.id_offsets[i]), int(self.id_offsets[i + 1])
        return bytes(self.id_bytes[a:b]).decode("utf-8")


class H5Store(ProteinStore):
    """The reference HDF5 layout (h5py when importable, else :class:`.hdf5.H5File` over mmap).

    Fixes the reference reader's defects: root-level datasets as E3 writes them, no
    removed ``Dataset.value`` API, a working ``__len__``."""

    def __init__(self, path: str, backend: str = "auto"):
        if backend == "auto":
            backend = "h5py" if h5py is not None else "pbx"
        self.backend = backend
        self.f = h5py.File(path, "r") if backend == "h5py" else pbx_h5.H5File(path)
        self.included_annotations = [_text(x) for x in self.f["included_annotations"][:]]
        self.n_annotations = len(self.included_annotations)
        self._seqs, self._ids, self._masks = self.f["seqs"], self.f["uniprot_ids"], self.f["annotation_masks"]

    def __len__(self) -> int:
        return int(self._seqs.shape[0])

    def seq(self, i: int) -> str:
        return _text(self._seqs[i])

    def annotation_mask(self, i: int) -> np.ndarray:
        return np.array(self._masks[i], dtype=bool)

    def uniprot_id(self, i: int) -> str:
        return _text(self._ids[i])

    def close(self) -> None:
        self.f.close()


class ProteinStoreWriter:
    """Chunked writer for the E3 layout (reference ``create_h5_dataset`` pass 2,
    ``uniref_dataset.py:249-268``).  ``fmt`` = ``pbxds`` | ``h5``.

    ``.pbxds`` records are streamed to raw side files as they arrive (only the per-record lengths
    stay in memory), then converted to ``.npy`` in bounded chunks on :meth:`close`, so a
    UniRef90-sized dataset is written in O(n) host memory of 16 B per record."""

    _CHUNK = 1 << 24

    def __init__(self, path: str, included_annotations: Sequence[str], fmt: str = "auto"):
        if fmt == "auto":
            fmt = "h5" if path.endswith((".h5", ".hdf5")) else "pbxds"
        self.path, self.fmt = path, fmt
        self.included_annotations = list(included_annotations)
        self.n_ann = len(self.included_annotations)
        self._nbytes = (self.n_ann + 7) // 8
        self._seq_lens: List[int] = []
        self._id_lens: List[int] = []
        if fmt == "pbxds":
            os.makedirs(path, exist_ok=True)
            self._fseq = open(os.path.join(path, "seq_bytes.raw"), "wb")
            self._fid = open(os.path.join(path, "id_bytes.raw"), "wb")
            self._fbits = open(os.path.join(path, "annotation_bits.raw"), "wb")
        else:  # streaming HDF5 writer (same layout h5py writes; no h5py needed)
            self._h5 = pbx_h5.H5Writer(path, self.included_annotations)

    def append(self, uniprot_id: str, seq: str, annotation_indices: Iterable[int]) -> None:
        mask = np.zeros(self.n_ann, dtype=bool)
        idx = np.fromiter((int(i) for i in annotation_indices), dtype=np.int64)
        if idx.size:
            mask[idx] = True
        self.append_mask(uniprot_id, seq, mask)

    def append_mask(self, uniprot_id: str, seq: str, mask: np.ndarray) -> None:
        uid, sq = uniprot_id.encode("utf-8"), seq.encode("ascii")
        bits = np.packbits(np.asarray(mask, dtype=bool)[:self.n_ann], bitorder="little")
        if bits.size < self._nbytes:
            bits = np.pad(bits, (0, self._nbytes - bits.size))
        self._seq_lens.append(len(sq))
        self._id_lens.append(len(uid))
        if self.fmt == "pbxds":
            self._fseq.write(sq)
            self._fid.write(uid)
            self._fbits.write(bits.tobytes())
        else:
            self._h5.append(uniprot_id, seq, bits)

    def __len__(self) -> int:
        return len(self._seq_lens)

    def close(self) -> None:
        if self.fmt == "pbxds":
            self._write_pbxds()
        else:
            self._h5.close()

    def _raw_to_npy(self, raw_name: str, npy_name: str, shape) -> None:
        raw = os.path.join(self.path, raw_name)
        out = np.lib.format.open_memmap(os.path.join(self.path, npy_name), mode="w+", dtype=np.uint8, shape=shape)
        flat = out.reshape(-1)
        with open(raw, "rb") as f:
            pos = 0
            while True:
                buf = f.read(self._CHUNK)
                if not buf:
                    break
                flat[pos:pos + len(buf)] = np.frombuffer(buf, dtype=np.uint8)
                pos += len(buf)
        if pos != flat.size:
            raise IOError(f"{raw}: wrote {pos} bytes, expected {flat.size}")
        out.flush()
        del out, flat
        os.remove(raw)

    def _write_pbxds(self) -> None:
        for fh in (self._fseq, self._fid, self._fbits):
            fh.close()
        n = len(self._seq_lens)
        lens = np.asarray(self._seq_lens, dtype=np.int64)
        offs = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        id_offs = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(np.asarray(self._id_lens, dtype=np.int64), out=id_offs[1:])
        sv = lambda name, arr: np.save(os.path.join(self.path, name), arr, allow_pickle=False)  # noqa: E731
        sv("seq_offsets.npy", offs)
        sv("seq_lengths.npy", lens.astype(np.int32))
        sv("id_offsets.npy", id_offs)
        self._raw_to_npy("seq_bytes.raw", "seq_bytes.npy", (int(offs[-1]),))
        self._raw_to_npy("id_bytes.raw", "id_bytes.npy", (int(id_offs[-1]),))
        self._raw_to_npy("annotation_bits.raw", "annotation_bits.npy", (n, self._nbytes))
        with open(os.path.join(self.path, "meta.json"), "w") as f:
            json.dump({"version": PBXDS_VERSION, "n": n, "n_annotations": self.n_ann,
                       "included_annotations": self.included_annotations}, f)
