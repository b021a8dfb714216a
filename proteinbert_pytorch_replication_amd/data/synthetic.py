"""Synthetic UniRef90/GO-shaped data, generated and corrupted on the device.

The reference's only data backend for its driver is
``create_random_samples`` (``ProteinBERT/dummy_tests.py:23-38``): lengths
``U[0, 250]``, 22 amino acids uniform, 8943 annotations each Bernoulli(0.005).
Per-sample Python corruption (``data_processing.py:159-180``) cannot feed a
GPU, so here a whole padded batch is produced in a handful of device ops
(or one fused HIP kernel, ``ops.corrupt``) with the same distributions:

* tokens: ``<sos> aa... <eos>``, random-cropped to L (reference crop quirk:
  the start is drawn from ``[0, n+2-L)``), padded with ``<pad>``;
* token corruption: Bernoulli(p) on non-special tokens, replacement
  ``U{3..25}``;
* annotation corruption: blank with probability 0.5, else
  ``(ann + Bern(neg)) * Bern(1 - pos)``;
* weights: ``w_local = token != <pad>``, ``w_global = any(ann)`` broadcast.
"""
from __future__ import annotations

import random
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

from .vocab import ALL_AMINO_ACIDS, PAD_ID, SOS_ID, EOS_ID, VOCAB_SIZE

Batch = Tuple[Dict[str, torch.Tensor], Dict[str, torch.Tensor], Dict[str, torch.Tensor]]


def create_random_samples(nb_samples: int, seed: int = 7777, num_annotations: int = 8943,
                          max_length: int = 250) -> List[Tuple[str, List[int]]]:
    """Same distribution and RNG stream as reference dummy_tests.py:23-38."""
    samples = []
    rnd = random.Random(seed)
    for _ in range(nb_samples):
        n = rnd.randint(0, max_length)
        seq = "".join(ALL_AMINO_ACIDS[rnd.randint(0, len(ALL_AMINO_ACIDS) - 1)] for _ in range(n))
        ann = [0 if rnd.random() * 1000 > 5 else 1 for _ in range(num_annotations)]
        samples.append((seq, ann))
    return samples


@dataclass
class CorruptionParams:
    token_p: float = 0.05
    positive_p: float = 0.25
    negative_p: float = 1e-4
    blank_p: float = 0.5


def corrupt_batch_torch(tokens: torch.Tensor, ann: torch.Tensor, params: CorruptionParams,
                        generator: Optional[torch.Generator] = None,
                        weights_dtype: torch.dtype = torch.float32) -> Batch:
    """Batched D3/D4 corruption + weights (torch ops; oracle for the HIP kernel)."""
    B = tokens.shape[0]
    dev = tokens.device
    r = torch.rand(tokens.shape, device=dev, generator=generator)
    mask = (r < params.token_p) & (tokens > EOS_ID)
    rnd_tok = torch.randint(3, VOCAB_SIZE, tokens.shape, device=dev, generator=generator)
    x_local = torch.where(mask, rnd_tok, tokens)
    blank = torch.rand((B, 1), device=dev, generator=generator) <= params.blank_p
    keep = torch.rand(ann.shape, device=dev, generator=generator) >= params.positive_p
    add = torch.rand(ann.shape, device=dev, generator=generator) < params.negative_p
    x_global = (ann + add.to(ann.dtype)) * keep.to(ann.dtype)
    x_global = torch.where(blank, torch.zeros_like(x_global), x_global)
    w_local = (tokens != PAD_ID).to(weights_dtype)
    w_global = (ann != 0).any(dim=1, keepdim=True).to(weights_dtype).expand_as(ann)
    return ({"local": x_local, "global": x_global},
            {"local": tokens, "global": ann},
            {"local": w_local, "global": w_global})


class SyntheticUniRefGO:
    """Generates padded clean batches ``(tokens[B,L], ann[B,A])`` on ``device``."""

    def __init__(self, seq_len: int, num_annotations: int = 8943, batch_size: int = 32,
                 device: torch.device | str = "cpu", min_length: int = 0,
                 max_length: Optional[int] = None, density: float = 0.005, seed: int = 0,
                 corruption: CorruptionParams = CorruptionParams(), use_kernel: Optional[bool] = None):
        self.L, self.A, self.B = seq_len, num_annotations, batch_size
        self.device = torch.device(device)
        self.min_length = min_length
        # Longer than L by default so that the crop path is exercised (paper
        # sequences are often longer than the training window).
        self.max_length = max_length if max_length is not None else seq_len + 64
        self.density = density
        self.corruption = corruption
        self.generator = torch.Generator(device=self.device)
        self.generator.manual_seed(seed)
        self.seed = seed
        self.step = 0
        self.gen_step = 0
        if use_kernel is None:
            use_kernel = self.device.type == "cuda"
        self.use_kernel = use_kernel
        # device-side step counter: generation launches read it, so a hipGraph-captured step draws a
        # fresh batch on every replay (the counter is advanced by a captured add)
        self.step_dev = torch.zeros(1, dtype=torch.int64, device=self.device) if use_kernel else None

    def clean_batch(self) -> Tuple[torch.Tensor, torch.Tensor]:
        B, L, dev, g = self.B, self.L, self.device, self.generator
        if self.use_kernel:
            from ..ops.corrupt import synth_batch
            return synth_batch(B, L, self.A, self.min_length, self.max_length, self.density, self.seed,
                               1, dev, step_dev=self.step_dev)
        n = torch.randint(self.min_length, self.max_length + 1, (B, 1), device=dev, generator=g)
        total = n + 2  # <sos> + aa + <eos>
        span = (total - L).clamp(min=1)
        # reference crop: start ~ randint(0, total - L) exclusive, only when total > L
        start = torch.where(total > L, (torch.rand((B, 1), device=dev, generator=g) * span).long(),
                            torch.zeros_like(total))
        s = start + torch.arange(L, device=dev).unsqueeze(0)
        aa = torch.randint(4, VOCAB_SIZE, (B, L), device=dev, generator=g)
        tok = torch.where(s == 0, torch.full_like(aa, SOS_ID), aa)
        tok = torch.where(s == total - 1, torch.full_like(aa, EOS_ID), tok)
        tok = torch.where(s >= total, torch.full_like(aa, PAD_ID), tok)
        ann = (torch.rand((B, self.A), device=dev, generator=g) < self.density).float()
        return tok, ann

    def corrupt(self, tokens: torch.Tensor, ann: torch.Tensor) -> Batch:
        if self.use_kernel:
            from ..ops import corrupt as corrupt_op
            out = corrupt_op.corrupt_batch(tokens, ann, self.corruption, seed=self.seed, step=1,
                                           step_dev=self.step_dev)
            if self.step_dev.is_cuda:
                from ..ops import _lib
                _lib.call("pbx_add_i64", self.step_dev.data_ptr(), 1, _lib.stream_ptr(self.step_dev.device))
            else:
                self.step_dev.add_(1)
            return out
        return corrupt_batch_torch(tokens, ann, self.corruption, self.generator)

    def __iter__(self):
        while True:
            yield self.next_batch()

    def next_batch(self) -> Batch:
        tok, ann = self.clean_batch()
        return self.corrupt(tok, ann)


class MultiLengthSynthetic:
    """Batches whose sequence length cycles through ``lengths`` (the paper trained on a mix of
    L = 128 / 512 / 1024; reference ``modules.py:148-151`` would need one model per L).  Pair with
    ``ProteinBERT(..., sequences_length=max(lengths), variable_length=True)``.  ``batch_sizes``: one
    per length (e.g. constant tokens per batch), default ``batch_size`` for all."""

    def __init__(self, lengths, num_annotations: int = 8943, batch_size: int = 32, device="cpu",
                 batch_sizes=None, seed: int = 0, **kw):
        self.lengths = [int(x) for x in lengths]
        bs = [int(b) for b in batch_sizes] if batch_sizes else [batch_size] * len(self.lengths)
        self.gens = [SyntheticUniRefGO(L, num_annotations, b, device, seed=seed + 7919 * i, **kw)
                     for i, (L, b) in enumerate(zip(self.lengths, bs))]
        self.i = 0

    def __iter__(self):
        while True:
            yield self.next_batch()

    def next_batch(self) -> Batch:
        g = self.gens[self.i % len(self.gens)]
        self.i += 1
        return g.next_batch()


class SyntheticSecondaryStructure(torch.utils.data.Dataset):
    """Per-residue labelled synthetic proteins for the fine-tuning path (BASELINE cfg 5).

    Item: ``(tokens int64 [L], labels int64 [L])``; labels are a fixed function of the residue
    window ``(x[i-1], x[i], x[i+1])`` (so a head on a contextual encoder can learn them), ``-100``
    on ``<sos>``/``<eos>``/``<pad>``.  ``n_classes`` 3 (H/E/C) or 8 (DSSP) by convention.
    """

    def __init__(self, n: int, seq_len: int, n_classes: int = 8, min_length: int = 16,
                 max_length: Optional[int] = None, seed: int = 0):
        g = torch.Generator().manual_seed(seed)
        L = seq_len
        max_length = max_length if max_length is not None else L - 2
        lens = torch.randint(min_length, max_length + 1, (n,), generator=g)
        aa = torch.randint(4, VOCAB_SIZE, (n, L), generator=g)
        pos = torch.arange(L).unsqueeze(0)
        tok = torch.where(pos == 0, torch.full_like(aa, SOS_ID), aa)
        tok = torch.where(pos == lens.unsqueeze(1) + 1, torch.full_like(aa, EOS_ID), tok)
        tok = torch.where(pos > lens.unsqueeze(1) + 1, torch.full_like(aa, PAD_ID), tok)
        prev = torch.roll(tok, 1, 1)
        nxt = torch.roll(tok, -1, 1)
        lab = (tok * 7 + prev * 3 + nxt * 5) % n_classes
        lab = torch.where(tok > EOS_ID, lab, torch.full_like(lab, -100))
        self.tokens, self.labels = tok, lab

    def __len__(self) -> int:
        return self.tokens.shape[0]

    def __getitem__(self, i: int):
        return self.tokens[i], self.labels[i]
