"""Per-sample host-side transforms with the reference's semantics.

Reference: ``ProteinBERT/data_processing.py:30-142``.  These are the CPU path
(used by the map-style datasets and as the oracle for the on-device
corruption in :mod:`.synthetic`).  Quirks are kept by default and can be
switched off:

* ``SentenceRandomCrop`` draws ``start ~ randint(0, len - max)`` with an
  exclusive high, so the last window is never chosen
  (``data_processing.py:82``); ``include_last_window=True`` fixes it.
* ``SimpleTokenRandomizer`` replaces with ``randint(3, V)`` which includes
  ``<unk>`` and may equal the original token (``:104-105``).
* ``AnnotationMasking`` blanks the whole vector with probability 0.5 and can
  produce the value 2.0 when a positive also receives a false positive
  (``:127-140``).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Union

import numpy as np
import torch

from .vocab import Vocab, PAD_ID, SOS_ID, EOS_ID


class SimpleCharacterTokenizer:
    """``list(seq)`` -> ids, optionally framed by ``<sos>``/``<eos>``."""

    def __init__(self, vocab: Vocab, add_sos_eos: bool = True, sos_index: int = SOS_ID,
                 eos_index: int = EOS_ID):
        assert isinstance(add_sos_eos, bool)
        self.vocab = vocab
        self.add_sos_eos = add_sos_eos
        self.sos_index = sos_index
        self.eos_index = eos_index

    def encode_np(self, sample: str) -> np.ndarray:
        ids = self.vocab.encode(sample)
        if self.add_sos_eos:
            ids = np.concatenate([[self.sos_index], ids, [self.eos_index]]).astype(np.int64)
        return ids

    def __call__(self, sample: str) -> List[int]:
        return self.encode_np(sample).tolist()


class SentenceRandomCrop:
    def __init__(self, max_length: int, include_last_window: bool = False,
                 generator: Optional[torch.Generator] = None):
        assert isinstance(max_length, int)
        self.max_length = max_length
        self.include_last_window = include_last_window
        self.generator = generator

    def start_index(self, length: int) -> int:
        hi = length - self.max_length + (1 if self.include_last_window else 0)
        return int(torch.randint(0, hi, (1,), generator=self.generator)[0])

    def __call__(self, sample):
        if len(sample) <= self.max_length:
            return sample
        s = self.start_index(len(sample))
        return sample[s:s + self.max_length]


class SimpleTokenRandomizer:
    def __init__(self, vocab: Union[Vocab, int], p: float = .05,
                 generator: Optional[torch.Generator] = None,
                 exclude_tokens: Sequence[int] = (PAD_ID, SOS_ID, EOS_ID)):
        assert isinstance(p, float)
        self.vocab_size = vocab if isinstance(vocab, int) else len(vocab)
        self.p = p
        self.exclude_tokens = tuple(exclude_tokens)
        self.generator = generator

    def __call__(self, sample: torch.Tensor) -> torch.Tensor:
        sample = torch.as_tensor(sample)
        mask = torch.rand(sample.shape, generator=self.generator) < self.p
        for t in self.exclude_tokens:
            mask &= sample != t
        rnd = torch.randint(3, self.vocab_size, sample.shape, generator=self.generator)
        return torch.where(mask, rnd, sample)


class AnnotationMasking:
    def __init__(self, positive_p: float = 0.25, negative_p: float = 0.0001,
                 blank_p: float = 0.5, generator: Optional[torch.Generator] = None):
        assert isinstance(positive_p, float)
        assert isinstance(negative_p, float)
        self.positive_p = positive_p
        self.negative_p = negative_p
        self.blank_p = blank_p
        self.generator = generator

    def __call__(self, sample) -> torch.Tensor:
        sample = torch.as_tensor(sample)
        if float(torch.rand(1, generator=self.generator)[0]) <= self.blank_p:
            return torch.zeros(sample.shape, dtype=sample.dtype)
        keep = (torch.rand(sample.shape, generator=self.generator) >= self.positive_p).to(sample.dtype)
        add = (torch.rand(sample.shape, generator=self.generator) < self.negative_p).to(sample.dtype)
        return (sample + add) * keep


def pad_to(ids: Union[np.ndarray, torch.Tensor, List[int]], length: int, pad_value: int = PAD_ID) -> torch.Tensor:
    t = torch.as_tensor(ids, dtype=torch.long)
    if t.numel() >= length:
        return t[:length]
    out = torch.full((length,), pad_value, dtype=torch.long)
    out[:t.numel()] = t
    return out
