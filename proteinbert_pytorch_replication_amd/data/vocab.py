"""Amino-acid vocabulary (no torchtext).

Same ids as the reference ``create_amino_acid_vocab`` (reference
``ProteinBERT/data_processing.py:337-348``): the four specials first, then the
22 amino-acid letters in alphabetical order; unknown characters map to
``<unk>``.  The ids are part of the checkpoint contract (embedding rows).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Sequence

import numpy as np

ALL_AMINO_ACIDS = "ACDEFGHIKLMNPQRSTUVWXY"
SPECIAL_TOKENS = ("<pad>", "<sos>", "<eos>", "<unk>")
PAD_ID, SOS_ID, EOS_ID, UNK_ID = 0, 1, 2, 3
VOCAB_SIZE = len(SPECIAL_TOKENS) + len(ALL_AMINO_ACIDS)  # 26


class Vocab:
    """Minimal string<->id table with a default index (``<unk>``)."""

    def __init__(self, tokens: Sequence[str], default_token: str = "<unk>"):
        self._itos: List[str] = list(tokens)
        self._stoi: Dict[str, int] = {t: i for i, t in enumerate(self._itos)}
        self.default_index = self._stoi[default_token]
        # 256-entry byte lookup table for fast numpy encoding of ASCII sequences
        lut = np.full(256, self.default_index, dtype=np.int64)
        for t, i in self._stoi.items():
            if len(t) == 1:
                lut[ord(t)] = i
        self.byte_lut = lut

    def __getitem__(self, token: str) -> int:
        return self._stoi.get(token, self.default_index)

    def __len__(self) -> int:
        return len(self._itos)

    def __contains__(self, token: str) -> bool:
        return token in self._stoi

    def get_itos(self) -> List[str]:
        return list(self._itos)

    def get_stoi(self) -> Dict[str, int]:
        return dict(self._stoi)

    def get_default_index(self) -> int:
        return self.default_index

    def lookup_indices(self, tokens: Iterable[str]) -> List[int]:
        return [self[t] for t in tokens]

    def lookup_token(self, index: int) -> str:
        return self._itos[index]

    def lookup_tokens(self, indices: Iterable[int]) -> List[str]:
        return [self._itos[i] for i in indices]

    def encode(self, seq: str) -> np.ndarray:
        """Vectorised character -> id (no specials added)."""
        raw = np.frombuffer(seq.encode("ascii", errors="replace"), dtype=np.uint8)
        return self.byte_lut[raw]

    def decode(self, ids: Iterable[int], strip_specials: bool = True) -> str:
        out = []
        for i in ids:
            i = int(i)
            if strip_specials and i < len(SPECIAL_TOKENS):
                continue
            out.append(self._itos[i] if len(self._itos[i]) == 1 else "?")
        return "".join(out)


def create_amino_acid_vocab() -> Vocab:
    """Same API name and ids as the reference (data_processing.py:337)."""
    return Vocab(list(SPECIAL_TOKENS) + list(ALL_AMINO_ACIDS))
