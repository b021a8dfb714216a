"""Dependency-free TensorBoard scalar writer (optional TensorBoard writer).

Neither ``tensorboard`` nor ``tensorflow`` is in this image, and ``torch.utils.tensorboard`` needs
the former, so the event file is written here directly:

* an event file is a TFRecord stream: ``uint64 length | uint32 masked_crc32c(length) | data |
  uint32 masked_crc32c(data)`` (little endian; CRC-32C, Castagnoli polynomial, masked as
  ``((c >> 15) | (c << 17)) + 0xa282ead8``);
* each record is a serialized ``tensorflow.Event`` protobuf, encoded by hand: ``wall_time`` (field 1,
  double), ``step`` (2, int64), ``file_version`` (3, string, the first record: ``brain.Event:2``) and
  ``summary`` (5, message ``Summary { repeated Value value = 1 }`` with ``Value { string tag = 1;
  float simple_value = 2 }``).

The reference logs loss / learning rate / iteration time with ``logging`` only
(``ProteinBERT/utils.py:308-313``); :func:`..train.pretrain.pretrain` writes the same quantities here
when given ``tensorboard_dir`` (rank 0).  :func:`read_scalars` parses a file back (tests, tooling).
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Dict, List, Optional, Tuple

_CRC_TABLE: List[int] = []


def _crc_table() -> List[int]:
    if not _CRC_TABLE:
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
            _CRC_TABLE.append(c)
    return _CRC_TABLE


def crc32c(data: bytes) -> int:
    t = _crc_table()
    c = 0xFFFFFFFF
    for b in data:
        c = t[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n: int) -> bytes:
    n &= (1 << 64) - 1                     # int64 fields: two's complement, 10 bytes when negative
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field_bytes(num: int, payload: bytes) -> bytes:
    return _varint((num << 3) | 2) + _varint(len(payload)) + payload


def _event(wall_time: float, step: Optional[int] = None, file_version: Optional[str] = None,
           summary: Optional[bytes] = None) -> bytes:
    out = bytearray(b"\x09" + struct.pack("<d", wall_time))              # field 1, fixed64
    if step is not None:
        out += b"\x10" + _varint(int(step))                                # field 2, varint
    if file_version is not None:
        out += _field_bytes(3, file_version.encode())
    if summary is not None:
        out += _field_bytes(5, summary)
    return bytes(out)


def _scalar_summary(tag: str, value: float) -> bytes:
    v = _field_bytes(1, tag.encode()) + b"\x15" + struct.pack("<f", float(value))   # Value.tag, .simple_value
    return _field_bytes(1, v)                                                        # Summary.value


def _record(data: bytes) -> bytes:
    header = struct.pack("<Q", len(data))
    return header + struct.pack("<I", masked_crc32c(header)) + data + struct.pack("<I", masked_crc32c(data))


class SummaryWriter:
    """``add_scalar(tag, value, step)`` into ``logdir/events.out.tfevents.<time>.<host>.pbx``."""

    def __init__(self, logdir: str, flush_every: int = 20):
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.pbx")
        self._f = open(self.path, "ab")
        self._f.write(_record(_event(time.time(), file_version="brain.Event:2")))
        self._n = 0
        self.flush_every = max(1, flush_every)

    def add_scalar(self, tag: str, value: float, step: int, wall_time: Optional[float] = None) -> None:
        self._f.write(_record(_event(time.time() if wall_time is None else wall_time, step=step,
                                     summary=_scalar_summary(tag, value))))
        self._n += 1
        if self._n % self.flush_every == 0:
            self._f.flush()

    def add_scalars(self, values: Dict[str, float], step: int) -> None:
        for k, v in values.items():
            self.add_scalar(k, v, step)

    def flush(self) -> None:
        self._f.flush()

    def close(self) -> None:
        if self._f is not None:
            self._f.close()
            self._f = None


# --- reader (tests / tooling) ----------------------------------------------------------------------
def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    shift = n = 0
    while True:
        x = b[i]
        i += 1
        n |= (x & 0x7F) << shift
        shift += 7
        if not x & 0x80:
            return n, i


def _parse_fields(b: bytes):
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 1:
            v, i = b[i:i + 8], i + 8
        elif wt == 5:
            v, i = b[i:i + 4], i + 4
        elif wt == 2:
            n, i = _read_varint(b, i)
            v, i = b[i:i + n], i + n
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield num, wt, v


def read_scalars(path: str) -> List[Tuple[int, str, float]]:
    """(step, tag, value) of every scalar in an event file; verifies both CRCs of every record."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        header = data[i:i + 8]
        (n,) = struct.unpack("<Q", header)
        if struct.unpack("<I", data[i + 8:i + 12])[0] != masked_crc32c(header):
            raise ValueError("bad length CRC")
        rec = data[i + 12:i + 12 + n]
        if struct.unpack("<I", data[i + 12 + n:i + 16 + n])[0] != masked_crc32c(rec):
            raise ValueError("bad data CRC")
        i += 16 + n
        step = 0
        summ = None
        for num, _, v in _parse_fields(rec):
            if num == 2:
                step = v
            elif num == 5:
                summ = v
        if summ is None:
            continue
        for num, _, val in _parse_fields(summ):
            if num != 1:
                continue
            tag, sv = None, None
            for fn, _, fv in _parse_fields(val):
                if fn == 1:
                    tag = fv.decode()
                elif fn == 2:
                    sv = struct.unpack("<f", fv)[0]
            out.append((step, tag, sv))
    return out
