"""Dependency-free HDF5 reader and streaming writer for the reference dataset layout.

The reference's canonical on-disk dataset is an HDF5 file written by h5py
(``ProteinBERT/uniref_dataset.py:236-245``) with five root-level datasets::

    included_annotations[n_ann]  vlen UTF-8 str      uniprot_ids[n]  vlen UTF-8 str
    seqs[n]                      vlen UTF-8 str      seq_lengths[n]  int32
    annotation_masks[n, n_ann]   bool (h5py: enum int8 {FALSE=0, TRUE=1})

h5py is not importable in this image (nor is libhdf5), so this module implements the part of
the HDF5 file format (spec version 3.0) that such files use, directly on ``mmap``:

* :class:`H5File` - reader: superblock v0-v3, version-1 and version-2 object headers (with
  continuation blocks), symbol-table groups (v1 B-tree + SNOD + local heap) and compact link
  messages, contiguous / compact / chunked (v1 B-tree index, deflate + shuffle filters) layouts,
  fixed-point, floating-point, fixed and variable-length strings, enums, and the global heap
  that holds variable-length data.  Datasets slice like numpy arrays along the first axis.
* :class:`H5Writer` - streaming writer producing what h5py's default ("earliest") file format
  produces for this layout: superblock v0, version-1 object headers, a symbol-table root group,
  contiguous datasets, variable-length strings in global heap collections.  Records are
  appended one at a time; the only per-record host memory is in temporary side files, so a
  UniRef90-sized dataset is written with bounded memory.

Compatibility with files written by the real HDF5 library is by construction from the format
specification; no HDF5 library exists in this image to cross-check against, so that parity is
unpinned (``tests/test_hdf5.py`` round-trips our own files and checks the encoded structures
byte by byte against the specification's field layouts).  Files with a user block (superblock at
512 or later, base address != 0) are refused rather than read at shifted offsets.
"""
from __future__ import annotations

import mmap
import os
import struct
import zlib
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

UNDEF = 0xFFFFFFFFFFFFFFFF
SIGNATURE = b"\x89HDF\r\n\x1a\n"


def _align8(n: int) -> int:
    return (n + 7) & ~7


# =================================================================================================
# datatypes
# =================================================================================================
class H5Type:
    """Decoded datatype message (the subset this module understands)."""

    def __init__(self, cls: int, size: int, **kw):
        self.cls = cls
        self.size = size
        self.__dict__.update(kw)

    def numpy_dtype(self) -> np.dtype:
        if self.cls == 0:  # fixed-point
            return np.dtype(("<" if self.order == 0 else ">") + ("i" if self.signed else "u") + str(self.size))
        if self.cls == 1:  # floating-point
            return np.dtype(("<" if self.order == 0 else ">") + "f" + str(self.size))
        if self.cls == 8:  # enum: values in the base type; a {FALSE, TRUE} enum is numpy bool (h5py)
            if sorted(self.members) == ["FALSE", "TRUE"] and self.base.size == 1:
                return np.dtype(bool)
            return self.base.numpy_dtype()
        if self.cls == 3:
            return np.dtype("S" + str(self.size))
        raise TypeError(f"no numpy dtype for HDF5 class {self.cls}")

    @property
    def is_vlen(self) -> bool:
        return self.cls == 9


def _decode_dtype(buf, off: int) -> Tuple[H5Type, int]:
    """Decode a datatype message at ``off``; returns (type, bytes consumed)."""
    b0 = buf[off]
    cls, version = b0 & 0x0F, b0 >> 4
    bits = buf[off + 1] | (buf[off + 2] << 8) | (buf[off + 3] << 16)
    size = struct.unpack_from("<I", buf, off + 4)[0]
    p = off + 8
    if cls == 0:  # fixed-point: bit offset, precision
        t = H5Type(0, size, order=bits & 1, signed=bool(bits & 8))
        return t, 8 + 4
    if cls == 1:  # floating point: 12 bytes of properties
        return H5Type(1, size, order=bits & 1), 8 + 12
    if cls == 3:  # fixed-length string
        return H5Type(3, size, pad=bits & 0xF, cset=(bits >> 4) & 0xF), 8
    if cls == 4:  # bitfield
        return H5Type(0, size, order=bits & 1, signed=False), 8 + 4
    if cls == 8:  # enum
        nmemb = bits & 0xFFFF
        base, used = _decode_dtype(buf, p)
        p += used
        names = []
        for _ in range(nmemb):
            end = bytes(buf[p:p + 4096]).index(b"\0")
            names.append(bytes(buf[p:p + end]).decode("utf-8"))
            p += end + 1 if version >= 3 else _align8(end + 1)
        vals = [bytes(buf[p + i * base.size:p + (i + 1) * base.size]) for i in range(nmemb)]
        p += nmemb * base.size
        return H5Type(8, size, base=base, members=names, values=vals), p - off
    if cls == 9:  # variable length: sequence (0) or string (1)
        base, used = _decode_dtype(buf, p)
        return H5Type(9, size, vtype=bits & 0xF, pad=(bits >> 4) & 0xF, cset=(bits >> 8) & 0xF,
                      base=base), 8 + used
    if cls == 6:  # compound: not needed by the layout; report the size so headers still parse
        return H5Type(6, size), 8
    raise NotImplementedError(f"HDF5 datatype class {cls} is not supported")


def _fixed_type(size: int, signed: bool) -> bytes:
    """Fixed-point little-endian datatype message body (version 1)."""
    return struct.pack("<B3sIHH", 0x10, bytes([0x08 if signed else 0x00, 0, 0]), size, 0, 8 * size)


def _vlen_str_type() -> bytes:
    """Variable-length UTF-8 string (h5py.string_dtype()): class 9, parent = unsigned char."""
    return struct.pack("<B3sI", 0x19, bytes([0x01, 0x01, 0x00]), 16) + _fixed_type(1, False)


def _bool_enum_type() -> bytes:
    """numpy bool as h5py stores it: enum over int8 {FALSE = 0, TRUE = 1} (version 1 encoding)."""
    names = b"".join(n + b"\0" * (_align8(len(n) + 1) - len(n)) for n in (b"FALSE", b"TRUE"))
    return struct.pack("<B3sI", 0x18, bytes([2, 0, 0]), 1) + _fixed_type(1, True) + names + bytes([0, 1])


# =================================================================================================
# reader
# =================================================================================================
class H5Dataset:
    def __init__(self, f: "H5File", name: str, shape: Tuple[int, ...], dtype: H5Type, layout: dict,
                 filters: List[Tuple[int, Tuple[int, ...]]]):
        self.file, self.name, self.shape, self.type, self.layout, self.filters = f, name, shape, dtype, layout, filters
        self._chunk_index: Optional[List[Tuple[Tuple[int, ...], int, int, int]]] = None
        self._raw_cache: Dict[int, np.ndarray] = {}

    def __len__(self) -> int:
        return self.shape[0] if self.shape else 1

    @property
    def dtype(self) -> np.dtype:
        return np.dtype(object) if self.type.is_vlen else self.type.numpy_dtype()

    # raw element bytes ------------------------------------------------------------------------
    def _row_bytes(self) -> int:
        n = 1
        for d in self.shape[1:]:
            n *= d
        return n * self.type.size

    def _raw_rows(self, start: int, stop: int) -> np.ndarray:
        """uint8 [stop - start, row bytes] of the stored (file-format) elements."""
        rb = self._row_bytes()
        lay = self.layout
        if stop <= start:
            return np.zeros((0, rb), np.uint8)
        if lay["class"] == 1:  # contiguous
            if lay["addr"] == UNDEF:  # never written: fill value (zeros)
                return np.zeros((stop - start, rb), np.uint8)
            a = lay["addr"] + start * rb
            # a bytes copy, not a view: a view would pin the mmap open
            return np.frombuffer(self.file.mm[a:a + (stop - start) * rb], np.uint8).reshape(stop - start, rb)
        if lay["class"] == 0:  # compact
            data = lay["data"]
            return np.frombuffer(data, np.uint8, (stop - start) * rb, start * rb).reshape(stop - start, rb)
        return self._chunked_rows(start, stop)

    def _chunks(self):
        if self._chunk_index is None:
            self._chunk_index = []
            self.file._walk_chunk_btree(self.layout["addr"], len(self.layout["dims"]), self._chunk_index)
            self._chunk_index.sort()
        return self._chunk_index

    def _chunk_data(self, addr: int, nbytes: int, mask: int) -> np.ndarray:
        raw = bytes(self.file.mm[addr:addr + nbytes])
        for i, (fid, cd) in reversed(list(enumerate(self.filters))):
            if mask & (1 << i):
                continue
            if fid == 1:
                raw = zlib.decompress(raw)
            elif fid == 2:  # shuffle: bytes of element k are stored plane by plane
                es = cd[0] if cd else self.type.size
                a = np.frombuffer(raw, np.uint8)
                n = a.size // es
                raw = a[:n * es].reshape(es, n).T.copy().tobytes() + a[n * es:].tobytes()
            elif fid == 3:  # fletcher32: drop the trailing checksum
                raw = raw[:-4]
            else:
                raise NotImplementedError(f"HDF5 filter {fid} is not supported")
        return np.frombuffer(raw, np.uint8)

    def _chunked_rows(self, start: int, stop: int) -> np.ndarray:
        dims = self.layout["dims"]          # chunk dims incl. the trailing element-size dim
        rank = len(self.shape)
        if rank == 0:
            raise NotImplementedError("scalar chunked dataset")
        out = np.zeros((stop - start,) + tuple(self.shape[1:]) + (self.type.size,), np.uint8)
        cshape = tuple(dims[:rank])
        for offs, addr, nbytes, mask in self._chunks():
            r0 = offs[0]
            if r0 >= stop or r0 + cshape[0] <= start:
                continue
            data = self._raw_cache.get(addr)
            if data is None:
                data = self._chunk_data(addr, nbytes, mask).reshape(cshape + (self.type.size,))
                if len(self._raw_cache) > 64:
                    self._raw_cache.clear()
                self._raw_cache[addr] = data
            a, b = max(start, r0), min(stop, r0 + cshape[0])
            src = [slice(a - r0, b - r0)]
            dst = [slice(a - start, b - start)]
            for k in range(1, rank):
                n = min(cshape[k], self.shape[k] - offs[k])
                src.append(slice(0, n))
                dst.append(slice(offs[k], offs[k] + n))
            out[tuple(dst)] = data[tuple(src)]
        return out.reshape(stop - start, -1)

    # decoded values --------------------------------------------------------------------------
    def read(self, start: int = 0, stop: Optional[int] = None):
        stop = len(self) if stop is None else min(stop, len(self))
        raw = self._raw_rows(start, stop)
        if self.type.is_vlen:
            desc = raw.reshape(-1).view(np.uint8).reshape(-1, 16)
            lens = desc[:, :4].copy().view("<u4").reshape(-1)
            addrs = desc[:, 4:12].copy().view("<u8").reshape(-1)
            idx = desc[:, 12:16].copy().view("<u4").reshape(-1)
            out = np.empty(len(lens), dtype=object)
            string = self.type.vtype == 1
            for i in range(len(lens)):
                # a zero-length value may carry a null heap ID (libhdf5 writes address 0): no heap read
                v = b"" if int(lens[i]) == 0 else \
                    self.file.heap_object(int(addrs[i]), int(idx[i]))[:int(lens[i]) * self.type.base.size]
                out[i] = v if string else np.frombuffer(v, self.type.base.numpy_dtype())
            return out.reshape((stop - start,) + tuple(self.shape[1:]))
        arr = raw.reshape(-1).view(self.type.numpy_dtype())
        return arr.reshape((stop - start,) + tuple(self.shape[1:]))

    def __getitem__(self, key):
        if isinstance(key, (int, np.integer)):
            i = int(key)
            if i < 0:
                i += len(self)
            if not 0 <= i < len(self):
                raise IndexError(i)
            return self.read(i, i + 1)[0]
        if isinstance(key, slice):
            a, b, s = key.indices(len(self))
            v = self.read(a, b) if a < b else self.read(0, 0)
            return v[::s] if s != 1 else v
        if key is Ellipsis or key == ():
            return self.read()
        raise TypeError(f"unsupported index {key!r}")


class H5File:
    """Read-only HDF5 file over ``mmap`` (root-level datasets; nested groups by path)."""

    def __init__(self, path: str):
        self.path = path
        self._fh = open(path, "rb")
        self.mm = mmap.mmap(self._fh.fileno(), 0, access=mmap.ACCESS_READ)
        self._heaps: Dict[int, Dict[int, Tuple[int, int]]] = {}
        base = self._find_superblock()
        ver = self.mm[base + 8]
        if ver in (0, 1):
            so, sl = self.mm[base + 13], self.mm[base + 14]
            if (so, sl) != (8, 8):
                raise NotImplementedError("only 8-byte offsets / lengths are supported")
            p = base + 24 + (4 if ver == 1 else 0)
            self.base_addr, _, _, _ = struct.unpack_from("<QQQQ", self.mm, p)
            ent = p + 32
            self.root = struct.unpack_from("<Q", self.mm, ent + 8)[0]
        elif ver in (2, 3):
            so, sl = self.mm[base + 9], self.mm[base + 10]
            if (so, sl) != (8, 8):
                raise NotImplementedError("only 8-byte offsets / lengths are supported")
            self.base_addr, _, _, self.root = struct.unpack_from("<QQQQ", self.mm, base + 12)
        else:
            raise NotImplementedError(f"superblock version {ver}")
        if self.base_addr != 0 or base != 0:
            # a user block shifts every file address by the base address; this reader resolves
            # addresses as absolute file offsets, so such files are refused instead of misread
            raise NotImplementedError(f"{path}: HDF5 user block / non-zero base address ({self.base_addr}, "
                                      f"superblock at {base}) is not supported")
        self._links = self._group_links(self.root)

    def _find_superblock(self) -> int:
        off = 0
        while off + 8 <= len(self.mm):
            if self.mm[off:off + 8] == SIGNATURE:
                return off
            off = 512 if off == 0 else off * 2
        raise ValueError(f"{self.path}: not an HDF5 file")

    def close(self) -> None:
        self.mm.close()
        self._fh.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # object headers ---------------------------------------------------------------------------
    def _messages(self, addr: int) -> List[Tuple[int, int, int]]:
        """[(type, data offset, size)] of an object header (v1 or v2, continuations followed)."""
        mm = self.mm
        out: List[Tuple[int, int, int]] = []
        if mm[addr:addr + 4] == b"OHDR":
            flags = mm[addr + 5]
            p = addr + 6 + (16 if flags & 0x20 else 0) + (4 if flags & 0x10 else 0)
            nsz = 1 << (flags & 3)
            size = int.from_bytes(mm[p:p + nsz], "little")
            p += nsz
            blocks = [(p, p + size)]
            track = bool(flags & 0x04)
            while blocks:
                s, e = blocks.pop(0)
                q = s
                while q + 4 <= e - 4 or (q + 4 <= e and mm[s - 4:s] != b"OCHK"):
                    if e - q < (6 if track else 4):
                        break
                    mt, ms = mm[q], struct.unpack_from("<H", mm, q + 1)[0]
                    q += 4 + (2 if track else 0)
                    if mt == 0x10:
                        ca, cl = struct.unpack_from("<QQ", mm, q)
                        blocks.append((ca + 4, ca + cl - 4))
                    elif mt != 0:
                        out.append((mt, q, ms))
                    q += ms
            return out
        # version 1: version, reserved, nmsgs(2), refcount(4), header size(4), pad to 8
        nmsg = struct.unpack_from("<H", mm, addr + 2)[0]
        hsize = struct.unpack_from("<I", mm, addr + 8)[0]
        blocks = [(addr + 16, addr + 16 + hsize)]
        seen = 0
        while blocks and seen < nmsg:
            s, e = blocks.pop(0)
            q = s
            while q + 8 <= e and seen < nmsg:
                mt, ms = struct.unpack_from("<HH", mm, q)
                q += 8
                seen += 1
                if mt == 0x10:
                    ca, cl = struct.unpack_from("<QQ", mm, q)
                    blocks.append((ca, ca + cl))
                elif mt != 0:
                    out.append((mt, q, ms))
                q += ms
        return out

    # groups ------------------------------------------------------------------------------------
    def _group_links(self, addr: int) -> Dict[str, int]:
        links: Dict[str, int] = {}
        for mt, q, ms in self._messages(addr):
            if mt == 0x11:  # symbol table: v1 B-tree + local heap
                bt, lh = struct.unpack_from("<QQ", self.mm, q)
                heap = self._local_heap(lh)
                self._walk_group_btree(bt, heap, links)
            elif mt == 0x06:  # link message (compact new-style group)
                name, target = self._link_message(q)
                if target is not None:
                    links[name] = target
            elif mt == 0x02:
                raise NotImplementedError("dense (fractal-heap) link storage is not supported")
        return links

    def _link_message(self, q: int) -> Tuple[str, Optional[int]]:
        mm = self.mm
        flags = mm[q + 1]
        p = q + 2
        ltype = 0
        if flags & 0x08:
            ltype = mm[p]
            p += 1
        if flags & 0x04:
            p += 8
        if flags & 0x10:
            p += 1
        nlen_size = 1 << (flags & 3)
        nlen = int.from_bytes(mm[p:p + nlen_size], "little")
        p += nlen_size
        name = bytes(mm[p:p + nlen]).decode("utf-8")
        p += nlen
        if ltype != 0:
            return name, None
        return name, struct.unpack_from("<Q", mm, p)[0]

    def _local_heap(self, addr: int) -> int:
        if self.mm[addr:addr + 4] != b"HEAP":
            raise ValueError("bad local heap signature")
        return struct.unpack_from("<Q", self.mm, addr + 24)[0]  # data segment address

    def _cstr(self, off: int) -> str:
        end = self.mm.find(b"\0", off)
        return bytes(self.mm[off:end]).decode("utf-8")

    def _walk_group_btree(self, addr: int, heap_data: int, links: Dict[str, int]) -> None:
        mm = self.mm
        if mm[addr:addr + 4] == b"SNOD":
            n = struct.unpack_from("<H", mm, addr + 6)[0]
            for i in range(n):
                e = addr + 8 + 40 * i
                name_off, ohdr = struct.unpack_from("<QQ", mm, e)
                links[self._cstr(heap_data + name_off)] = ohdr
            return
        if mm[addr:addr + 4] != b"TREE" or mm[addr + 4] != 0:
            raise ValueError("bad group B-tree node")
        used = struct.unpack_from("<H", mm, addr + 6)[0]
        p = addr + 24
        for i in range(used):
            child = struct.unpack_from("<Q", mm, p + 8 + 16 * i)[0]
            self._walk_group_btree(child, heap_data, links)

    def _walk_chunk_btree(self, addr: int, ndims: int, out: list) -> None:
        mm = self.mm
        if mm[addr:addr + 4] != b"TREE" or mm[addr + 4] != 1:
            raise ValueError("bad chunk B-tree node")
        level = mm[addr + 5]
        used = struct.unpack_from("<H", mm, addr + 6)[0]
        ksize = 8 + 8 * ndims
        p = addr + 24
        for i in range(used):
            k = p + i * (ksize + 8)
            nbytes, mask = struct.unpack_from("<II", mm, k)
            offs = struct.unpack_from("<" + "Q" * ndims, mm, k + 8)
            child = struct.unpack_from("<Q", mm, k + ksize)[0]
            if level == 0:
                out.append((tuple(offs[:-1]), child, nbytes, mask))
            else:
                self._walk_chunk_btree(child, ndims, out)

    # datasets ----------------------------------------------------------------------------------
    def keys(self) -> List[str]:
        return sorted(self._links)

    def __contains__(self, name: str) -> bool:
        try:
            self._resolve(name)
            return True
        except KeyError:
            return False

    def _resolve(self, name: str) -> int:
        links = self._links
        parts = [p for p in name.split("/") if p]
        addr = self.root
        for k, part in enumerate(parts):
            if part not in links:
                raise KeyError(name)
            addr = links[part]
            if k + 1 < len(parts):
                links = self._group_links(addr)
        return addr

    def __getitem__(self, name: str) -> H5Dataset:
        addr = self._resolve(name)
        shape, dtype, layout, filters = None, None, None, []
        for mt, q, ms in self._messages(addr):
            if mt == 0x01:
                shape = self._dataspace(q)
            elif mt == 0x03:
                dtype, _ = _decode_dtype(self.mm, q)
            elif mt == 0x08:
                layout = self._layout(q, ms)
            elif mt == 0x0B:
                filters = self._filters(q)
        if shape is None or dtype is None or layout is None:
            raise KeyError(f"{name} is not a dataset")
        return H5Dataset(self, name, shape, dtype, layout, filters)

    def _dataspace(self, q: int) -> Tuple[int, ...]:
        mm = self.mm
        ver, rank, flags = mm[q], mm[q + 1], mm[q + 2]
        if ver == 1:
            p = q + 8
        elif ver == 2:
            if mm[q + 3] == 2:  # null dataspace
                return (0,)
            p = q + 4
        else:
            raise NotImplementedError(f"dataspace version {ver}")
        return tuple(struct.unpack_from("<" + "Q" * rank, mm, p)) if rank else ()

    def _layout(self, q: int, ms: int) -> dict:
        mm = self.mm
        ver = mm[q]
        if ver != 3:
            raise NotImplementedError(f"data layout message version {ver}")
        cls = mm[q + 1]
        if cls == 0:
            n = struct.unpack_from("<H", mm, q + 2)[0]
            return {"class": 0, "data": bytes(mm[q + 4:q + 4 + n])}
        if cls == 1:
            a, s = struct.unpack_from("<QQ", mm, q + 2)
            return {"class": 1, "addr": a, "size": s}
        if cls == 2:
            nd = mm[q + 2]
            a = struct.unpack_from("<Q", mm, q + 3)[0]
            dims = struct.unpack_from("<" + "I" * nd, mm, q + 11)
            return {"class": 2, "addr": a, "dims": dims}
        raise NotImplementedError(f"layout class {cls}")

    def _filters(self, q: int) -> List[Tuple[int, Tuple[int, ...]]]:
        mm = self.mm
        ver, n = mm[q], mm[q + 1]
        p = q + (8 if ver == 1 else 2)
        out = []
        for _ in range(n):
            fid = struct.unpack_from("<H", mm, p)[0]
            if ver == 1 or fid >= 256:
                nlen, fl, nv = struct.unpack_from("<HHH", mm, p + 2)
                p += 8 + (_align8(nlen) if ver == 1 else nlen)
            else:
                fl, nv = struct.unpack_from("<HH", mm, p + 2)
                p += 6
            cd = struct.unpack_from("<" + "I" * nv, mm, p)
            p += 4 * nv + (4 if ver == 1 and nv % 2 else 0)
            out.append((fid, cd))
        return out

    # global heap -------------------------------------------------------------------------------
    def heap_object(self, coll: int, idx: int) -> bytes:
        table = self._heaps.get(coll)
        if table is None:
            table = self._parse_collection(coll)
            if len(self._heaps) > 4096:
                self._heaps.clear()
            self._heaps[coll] = table
        off, size = table[idx]
        return bytes(self.mm[off:off + size])

    def _parse_collection(self, addr: int) -> Dict[int, Tuple[int, int]]:
        mm = self.mm
        if mm[addr:addr + 4] != b"GCOL":
            raise ValueError("bad global heap collection signature")
        csize = struct.unpack_from("<Q", mm, addr + 8)[0]
        end = addr + csize
        p = addr + 16
        table: Dict[int, Tuple[int, int]] = {}
        while p + 16 <= end:
            idx, _refs = struct.unpack_from("<HH", mm, p)
            size = struct.unpack_from("<Q", mm, p + 8)[0]
            if idx == 0:
                break
            table[idx] = (p + 16, size)
            p += 16 + _align8(size)
        return table


# =================================================================================================
# writer
# =================================================================================================
class _Collections:
    """Streams variable-length values into global heap collections (``GCOL``)."""

    TARGET = 1 << 20
    MAX_OBJECTS = 65000

    def __init__(self, fh, start: int):
        self.fh = fh
        self.pos = start            # file offset of the next collection
        self._objs: List[bytes] = []
        self._bytes = 16

    def add(self, value: bytes) -> Tuple[int, int]:
        """Returns (collection address, object index) the value will live at."""
        need = 16 + _align8(len(value))
        if self._objs and (self._bytes + need > self.TARGET or len(self._objs) >= self.MAX_OBJECTS):
            self.flush()
        self._objs.append(value)
        self._bytes += need
        return self.pos, len(self._objs)

    def flush(self) -> None:
        if not self._objs:
            return
        size = max(4096, self._bytes)
        out = bytearray(b"GCOL" + bytes([1, 0, 0, 0]) + struct.pack("<Q", size))
        for i, v in enumerate(self._objs, 1):
            out += struct.pack("<HHIQ", i, 1, 0, len(v)) + v + b"\0" * (_align8(len(v)) - len(v))
        free = size - len(out)
        if free >= 16:
            out += struct.pack("<HHIQ", 0, 0, 0, free) + b"\0" * (free - 16)
        else:
            out += b"\0" * free
        self.fh.seek(self.pos)
        self.fh.write(out)
        self.pos += size
        self._objs = []
        self._bytes = 16


class H5Writer:
    """Streaming writer of the reference dataset layout (see module docstring).

    ``append(uniprot_id, seq, mask)`` per record, then ``close()``.  Sequences and ids go into
    global heap collections as they arrive; their 16-byte vlen descriptors and the bit-packed
    annotation masks are streamed to side files and laid out as contiguous datasets on close."""

    def __init__(self, path: str, included_annotations: Sequence[str]):
        self.path = path
        self.ann = [str(a) for a in included_annotations]
        self.n_ann = len(self.ann)
        self._nb = (self.n_ann + 7) // 8
        self.n = 0
        self.fh = open(path, "w+b")
        self.fh.write(b"\0" * 96)                      # superblock, patched on close
        self.heap = _Collections(self.fh, 96)
        self._side = {k: open(f"{path}.{k}.tmp", "w+b") for k in ("ids", "seqs", "lens", "bits")}

    @staticmethod
    def _desc(n: int, where: Tuple[int, int]) -> bytes:
        return struct.pack("<IQI", n, where[0], where[1])

    def append(self, uniprot_id: str, seq: str, mask) -> None:
        uid, sq = uniprot_id.encode("utf-8"), seq.encode("utf-8")
        self._side["ids"].write(self._desc(len(uid), self.heap.add(uid)))
        self._side["seqs"].write(self._desc(len(sq), self.heap.add(sq)))
        self._side["lens"].write(struct.pack("<i", len(seq)))
        m = np.asarray(mask)
        if m.dtype == np.uint8 and m.size == self._nb:   # already bit-packed (little bit order)
            bits = m
        else:
            bits = np.packbits(m.astype(bool)[:self.n_ann], bitorder="little")
            if bits.size < self._nb:
                bits = np.pad(bits, (0, self._nb - bits.size))
        self._side["bits"].write(bits.tobytes())
        self.n += 1

    # ------------------------------------------------------------------------------------------
    def _copy_side(self, key: str) -> Tuple[int, int]:
        src = self._side[key]
        src.flush()
        size = src.tell()
        addr = self._end
        self.fh.seek(addr)
        src.seek(0)
        while True:
            buf = src.read(1 << 24)
            if not buf:
                break
            self.fh.write(buf)
        self._end = _align8(addr + size)
        return addr, size

    def _write_masks(self) -> Tuple[int, int]:
        src = self._side["bits"]
        src.flush()
        src.seek(0)
        addr = self._end
        self.fh.seek(addr)
        rows = max(1, (1 << 24) // max(1, self._nb))
        left = self.n
        while left:
            k = min(rows, left)
            packed = np.frombuffer(src.read(k * self._nb), np.uint8).reshape(k, self._nb)
            self.fh.write(np.unpackbits(packed, axis=1, bitorder="little")[:, :self.n_ann].tobytes())
            left -= k
        size = self.n * self.n_ann
        self._end = _align8(addr + size)
        return addr, size

    def _put(self, blob: bytes) -> int:
        addr = self._end
        self.fh.seek(addr)
        self.fh.write(blob)
        self._end = _align8(addr + len(blob))
        return addr

    @staticmethod
    def _msg(mtype: int, body: bytes, flags: int = 0) -> bytes:
        body = body + b"\0" * (_align8(len(body)) - len(body))
        return struct.pack("<HHB3x", mtype, len(body), flags) + body

    def _object_header(self, msgs: List[bytes]) -> bytes:
        payload = b"".join(msgs)
        return struct.pack("<BBHII", 1, 0, len(msgs), 1, len(payload)) + b"\0" * 4 + payload

    def _dataset(self, shape: Tuple[int, ...], dtype: bytes, addr: int, size: int) -> int:
        rank = len(shape)
        space = struct.pack("<BBBB4x", 1, rank, 1, 0) + struct.pack("<" + "Q" * rank, *shape) * 2
        fill = bytes([2, 2, 2, 0])                      # v2: alloc late, write if set, undefined
        if size == 0:
            addr = UNDEF
        layout = struct.pack("<BBQQ", 3, 1, addr, size)
        msgs = [self._msg(0x01, space), self._msg(0x03, dtype, 1), self._msg(0x05, fill, 1),
                self._msg(0x08, layout)]
        return self._put(self._object_header(msgs))

    def close(self) -> None:
        # included annotation names, then every collection is final
        ann_desc = b"".join(self._desc(len(a.encode()), self.heap.add(a.encode())) for a in self.ann)
        self.heap.flush()
        self._end = _align8(self.heap.pos)
        ann_addr = self._put(ann_desc) if ann_desc else 0
        ids_addr, ids_size = self._copy_side("ids")
        seq_addr, seq_size = self._copy_side("seqs")
        len_addr, len_size = self._copy_side("lens")
        msk_addr, msk_size = self._write_masks()
        n = self.n
        objs = {
            "annotation_masks": self._dataset((n, self.n_ann), _bool_enum_type(), msk_addr, msk_size),
            "included_annotations": self._dataset((self.n_ann,), _vlen_str_type(), ann_addr, len(ann_desc)),
            "seq_lengths": self._dataset((n,), _fixed_type(4, True), len_addr, len_size),
            "seqs": self._dataset((n,), _vlen_str_type(), seq_addr, seq_size),
            "uniprot_ids": self._dataset((n,), _vlen_str_type(), ids_addr, ids_size),
        }
        root = self._root_group(objs)
        eof = self._end
        self.fh.seek(eof)
        self.fh.truncate(eof)
        sb = SIGNATURE + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack("<HHI", 4, 16, 0)
        sb += struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
        sb += root
        self.fh.seek(0)
        self.fh.write(sb)
        self.fh.close()
        for k, fh in self._side.items():
            fh.close()
            os.remove(f"{self.path}.{k}.tmp")

    def _root_group(self, objs: Dict[str, int]) -> bytes:
        names = sorted(objs)
        # local heap data segment: "" at offset 0, then the names (8-byte aligned)
        data = bytearray(b"\0" * 8)
        offs = {}
        for nm in names:
            offs[nm] = len(data)
            enc = nm.encode()
            data += enc + b"\0" * (_align8(len(enc) + 1) - len(enc))
        free = 0
        if len(data) % 8 == 0:
            data += b"\0" * 16                         # a free block (list head), as the library keeps
            free = len(data) - 16
            data[free:free + 16] = struct.pack("<QQ", 1, 16)
        heap_data = self._put(bytes(data))
        heap = self._put(b"HEAP" + bytes([0, 0, 0, 0]) + struct.pack("<QQQ", len(data), free, heap_data))
        # one symbol table node with 2K = 8 entries (leaf K = 4)
        k2 = max(8, len(names))
        snod = bytearray(b"SNOD" + bytes([1, 0]) + struct.pack("<H", len(names)))
        for nm in names:
            snod += struct.pack("<QQII16x", offs[nm], objs[nm], 0, 0)
        snod += b"\0" * (40 * (k2 - len(names)))
        snod_addr = self._put(bytes(snod))
        # v1 B-tree group node: keys are heap offsets (key 0 = "", key 1 = the last name)
        tree = b"TREE" + bytes([0, 0]) + struct.pack("<HQQ", 1, UNDEF, UNDEF)
        tree += struct.pack("<QQQ", 0, snod_addr, offs[names[-1]] if names else 0)
        tree += b"\0" * (16 * 2 * 16)                   # room for 2K internal entries (K = 16)
        tree_addr = self._put(tree)
        ohdr = self._put(self._object_header([self._msg(0x11, struct.pack("<QQ", tree_addr, heap))]))
        # root symbol table entry: cache type 1 carries the B-tree / heap addresses
        return struct.pack("<QQII", 0, ohdr, 1, 0) + struct.pack("<QQ", tree_addr, heap)


def write_reference_h5(path: str, included_annotations: Sequence[str],
                       records: Iterable[Tuple[str, str, np.ndarray]]) -> int:
    """Write ``(uniprot_id, seq, mask)`` records in the reference layout; returns the count."""
    w = H5Writer(path, included_annotations)
    for uid, seq, mask in records:
        w.append(uid, seq, mask)
    w.close()
    return w.n
