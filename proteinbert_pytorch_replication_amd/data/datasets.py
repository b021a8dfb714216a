"""Map-style pretraining datasets producing the reference's ``(X, Y, W)`` triple.

Reference: ``UniRefGO_PretrainingDataset`` (``ProteinBERT/data_processing.py:146-183``)
and the (non-functional) ``UniRefGO_HDF5PretrainingDataset`` (``:186-333``).

Item layout (``data_processing.py:178-180``)::

    X = {"local": int64[L] corrupted tokens,  "global": f32[A] corrupted annotations}
    Y = {"local": int64[L] clean tokens,      "global": f32[A] clean annotations}
    W = {"local": w[L] = (Y_local != <pad>),  "global": w[A] = any(Y_global) repeated}

The weights are float64 in the reference (numpy ``astype(float)``), which
promotes the reference loss to float64; ``weights_dtype`` keeps that by
default for parity and can be set to float32.
"""
from __future__ import annotations

from typing import Any, Dict, Optional, Sequence, Tuple

import numpy as np
import torch
from torch.utils import data

from .vocab import create_amino_acid_vocab, PAD_ID
from .transforms import (SimpleCharacterTokenizer, SentenceRandomCrop, SimpleTokenRandomizer,
                         AnnotationMasking, pad_to)
from .store import ProteinStore

Triple = Tuple[Dict[str, torch.Tensor], Dict[str, torch.Tensor], Dict[str, torch.Tensor]]


class _PretrainItemBuilder:
    def __init__(self, seq_max_length: int, token_p: float = .05, positive_p: float = .25,
                 negative_p: float = 1e-4, weights_dtype: torch.dtype = torch.float64,
                 include_last_window: bool = False, generator: Optional[torch.Generator] = None):
        self.vocab = create_amino_acid_vocab()
        self.seq_max_length = seq_max_length
        self.tokenizer = SimpleCharacterTokenizer(self.vocab)
        self.crop = SentenceRandomCrop(seq_max_length, include_last_window, generator)
        self.token_randomizer = SimpleTokenRandomizer(self.vocab, p=float(token_p), generator=generator)
        self.annotations_masking = AnnotationMasking(positive_p=float(positive_p),
                                                     negative_p=float(negative_p), generator=generator)
        self.weights_dtype = weights_dtype

    def build(self, seq_str: str, ann: Any) -> Triple:
        L = self.seq_max_length
        seq = torch.as_tensor(self.crop(self.tokenizer.encode_np(seq_str)), dtype=torch.long)
        masked_seq = pad_to(self.token_randomizer(seq), L)
        seq = pad_to(seq, L)
        ann_t = torch.as_tensor(np.asarray(ann), dtype=torch.float32)
        masked_ann = self.annotations_masking(ann_t).float()
        seq_w = (seq != PAD_ID).to(self.weights_dtype)
        ann_w = torch.full(ann_t.shape, float(bool(ann_t.any())), dtype=self.weights_dtype)
        return ({"local": masked_seq, "global": masked_ann},
                {"local": seq, "global": ann_t},
                {"local": seq_w, "global": ann_w})


class UniRefGO_PretrainingDataset(data.Dataset):
    """DataFrame-backed dataset: column 0 = sequence string, column 1 = list[A] of 0/1."""

    def __init__(self, df, seq_max_length: int = 128, **kw):
        self.df = df
        self.builder = _PretrainItemBuilder(seq_max_length, **kw)
        self.vocab = self.builder.vocab

    def __getitem__(self, index: int) -> Triple:
        return self.builder.build(self.df.iloc[index, 0], self.df.iloc[index, 1])

    def __len__(self) -> int:
        return len(self.df.index)


class UniRefGO_StorePretrainingDataset(data.Dataset):
    """Dataset over the on-disk E3 layout (``seqs``, ``seq_lengths``,
    ``annotation_masks``, ``uniprot_ids``, ``included_annotations``).

    Replaces the reference's broken HDF5 reader: it reads the
    layout that the reference writer actually produces
    (``uniref_dataset.py:236-245``), through :class:`ProteinStore` (the reference HDF5
    file, or the memory-mapped ``.pbxds`` directory format).  ``rank``/``world_size`` shard the index space for DP.
    """

    def __init__(self, path: str, seq_max_length: int = 128, rank: int = 0, world_size: int = 1, **kw):
        self.store = ProteinStore.open(path)
        self.builder = _PretrainItemBuilder(seq_max_length, **kw)
        self.vocab = self.builder.vocab
        n = len(self.store)
        self.indices = np.arange(rank, n, world_size)

    def __getitem__(self, index: int) -> Triple:
        i = int(self.indices[index])
        return self.builder.build(self.store.seq(i), self.store.annotation_mask(i))

    def __len__(self) -> int:
        return len(self.indices)


# Reference-compatible alias; the store opens the reference's HDF5 files (with or without h5py).
UniRefGO_HDF5PretrainingDataset = UniRefGO_StorePretrainingDataset


def collate_triples(items: Sequence[Triple]) -> Triple:
    out = []
    for k in range(3):
        out.append({key: torch.stack([it[k][key] for it in items]) for key in ("local", "global")})
    return tuple(out)  # type: ignore[return-value]
