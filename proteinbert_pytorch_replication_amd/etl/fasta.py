"""Indexed FASTA access (the role pyfaidx.Faidx plays in reference ``uniref_dataset.py:299-314``).

Reads/writes the samtools ``.fai`` index (name, length, offset, line bases, line bytes) and fetches
whole records by seeking, so multi-GB UniRef90 FASTA files are never loaded into memory.
"""
from __future__ import annotations

import os
from typing import Dict, Iterator, NamedTuple, Tuple


class FaiEntry(NamedTuple):
    rlen: int
    offset: int
    lenc: int   # bases per line
    lenb: int   # bytes per line (incl. newline)


class FastaIndex:
    def __init__(self, fasta_path: str, build_index: bool = True):
        self.path = fasta_path
        self.fai_path = fasta_path + ".fai"
        if not os.path.exists(self.fai_path):
            if not build_index:
                raise FileNotFoundError(self.fai_path)
            self.build()
        self.index: Dict[str, FaiEntry] = {}
        with open(self.fai_path) as f:
            for line in f:
                name, rlen, off, lenc, lenb = line.rstrip("\n").split("\t")[:5]
                self.index[name] = FaiEntry(int(rlen), int(off), int(lenc), int(lenb))
        self._fh = open(self.path, "rb")

    def build(self) -> None:
        rows = []
        with open(self.path, "rb") as f:
            name = None
            rlen = offset = lenc = lenb = 0
            pos = 0
            for raw in f:
                if raw.startswith(b">"):
                    if name is not None:
                        rows.append((name, rlen, offset, lenc, lenb))
                    name = raw[1:].split()[0].decode()
                    rlen, lenc, lenb = 0, 0, 0
                    offset = pos + len(raw)
                else:
                    seq = raw.rstrip(b"\r\n")
                    if lenc == 0:
                        lenc, lenb = len(seq), len(raw)
                    rlen += len(seq)
                pos += len(raw)
            if name is not None:
                rows.append((name, rlen, offset, lenc, lenb))
        with open(self.fai_path, "w") as out:
            for r in rows:
                out.write("%s\t%d\t%d\t%d\t%d\n" % r)

    def __contains__(self, name: str) -> bool:
        return name in self.index

    def fetch(self, name: str, start: int = 1, end: int = None) -> str:
        """1-based inclusive [start, end] (pyfaidx ``fetch`` convention); KeyError when absent."""
        e = self.index[name]
        end = e.rlen if end is None else min(end, e.rlen)
        if start < 1 or start > end:
            return ""
        s0 = start - 1
        if e.lenc == 0:
            return ""
        first_byte = e.offset + (s0 // e.lenc) * e.lenb + s0 % e.lenc
        last = end - 1
        last_byte = e.offset + (last // e.lenc) * e.lenb + last % e.lenc
        self._fh.seek(first_byte)
        raw = self._fh.read(last_byte - first_byte + 1)
        return raw.replace(b"\n", b"").replace(b"\r", b"").decode("ascii")

    def __iter__(self) -> Iterator[Tuple[str, str]]:
        for name in self.index:
            yield name, self.fetch(name)

    def close(self) -> None:
        self._fh.close()
