"""Pretraining data-loader factory and loader throughput probe.

Reference: ``create_pretrain_dataloaders`` (``ProteinBERT/utils.py:71-107``, T4) and
``optimal_num_workers_testing`` (``utils.py:30-68``, T5).

* ``create_pretrain_dataloaders(train_dir, batch_size, recursive_dir, num_workers, ...)`` finds the
  dataset store(s) under ``train_dir`` (``.pbxds`` directories; ``.h5`` files in the reference
  layout, read by h5py or ``data/hdf5.py``) and returns a rank-sharded loader: the native C++ batch builder
  (:class:`..data.native_loader.NativeStoreLoader`, ``num_workers`` = builder threads) for
  ``.pbxds``, otherwise a ``torch.utils.data.DataLoader`` over the store dataset with a
  :class:`..parallel.sampler.ShardedSampler`.  Several stores are chained per epoch.
* ``optimal_num_workers_testing(dataset_or_path)`` times two epochs per worker/thread count and
  returns the timings; the reference's loop always passed ``num_workers=1`` (``utils.py:60-61``),
  this one really varies it.
"""
from __future__ import annotations

import glob
import os
import time
from typing import Dict, Iterator, List, Optional, Sequence, Union

import torch
from torch.utils.data import DataLoader, Dataset

from ..data.datasets import UniRefGO_StorePretrainingDataset, collate_triples
from ..data.native_loader import NativeStoreLoader, native_loader_available
from ..parallel import dist as pdist
from ..parallel.sampler import ShardedSampler


def find_stores(train_dir: str, recursive_dir: bool = False) -> List[str]:
    if os.path.isdir(train_dir) and os.path.exists(os.path.join(train_dir, "meta.json")):
        return [train_dir]
    if os.path.isfile(train_dir):
        return [train_dir]
    pats = ["*.pbxds", "*.h5", "*.hdf5"]
    out: List[str] = []
    for pat in pats:
        out += glob.glob(os.path.join(train_dir, "**", pat) if recursive_dir else os.path.join(train_dir, pat),
                         recursive=recursive_dir)
    out = sorted(p for p in out if not p.endswith(".pbxds") or os.path.exists(os.path.join(p, "meta.json")))
    if not out:
        raise FileNotFoundError(f"no dataset store under {train_dir} (recursive={recursive_dir})")
    return out


class ChainedLoader:
    """Iterates several loaders back to back (one epoch = one pass over every store)."""

    def __init__(self, loaders: Sequence):
        self.loaders = list(loaders)
        self._pos = 0

    def __len__(self) -> int:
        return sum(len(x) for x in self.loaders)

    def __iter__(self) -> Iterator:
        for ld in self.loaders:
            yield from ld

    def state_dict(self) -> Dict:
        return {"stores": [ld.state_dict() if hasattr(ld, "state_dict") else {} for ld in self.loaders]}

    def load_state_dict(self, st: Dict) -> None:
        for ld, s in zip(self.loaders, st.get("stores", [])):
            if s and hasattr(ld, "load_state_dict"):
                ld.load_state_dict(s)

    def close(self) -> None:
        for ld in self.loaders:
            if hasattr(ld, "close"):
                ld.close()


def create_pretrain_dataloaders(train_dir: str, batch_size: int, recursive_dir: bool = False, num_workers: int = 0,
                                seq_max_length: int = 512, device=None, shuffle: bool = True, seed: int = 0,
                                drop_last: bool = True, native: Optional[bool] = None, rank: Optional[int] = None,
                                world_size: Optional[int] = None):
    info = pdist.get_info()
    rank = info.rank if rank is None else rank
    world_size = info.world_size if world_size is None else world_size
    device = torch.device(device) if device is not None else info.device
    loaders = []
    for path in find_stores(train_dir, recursive_dir):
        use_native = path.endswith(".pbxds") or os.path.isdir(path)
        if native is not None:
            use_native = use_native and native
        if use_native and native_loader_available():
            loaders.append(NativeStoreLoader(path, batch_size, seq_max_length, device=device, rank=rank,
                                             world_size=world_size, shuffle=shuffle, seed=seed,
                                             drop_last=drop_last, num_threads=max(1, num_workers)))
        else:
            ds = UniRefGO_StorePretrainingDataset(path, seq_max_length=seq_max_length,
                                                  weights_dtype=torch.float32)
            sampler = ShardedSampler(len(ds), rank, world_size, shuffle=shuffle, seed=seed)
            loaders.append(DataLoader(ds, batch_size=batch_size, sampler=sampler, num_workers=num_workers,
                                      pin_memory=device.type == "cuda", drop_last=drop_last,
                                      collate_fn=collate_triples, persistent_workers=num_workers > 0))
    return loaders[0] if len(loaders) == 1 else ChainedLoader(loaders)


def optimal_num_workers_testing(dataset: Union[Dataset, str], batch_size: int = 64, epochs: int = 2,
                                worker_counts: Optional[Sequence[int]] = None, seq_max_length: int = 512,
                                max_batches: Optional[int] = None, verbose: bool = True) -> Dict[int, float]:
    """Seconds for ``epochs`` passes per worker count (threads for a ``.pbxds`` path)."""
    if worker_counts is None:
        worker_counts = [0, 1] + list(range(2, (os.cpu_count() or 2), 2))
    out: Dict[int, float] = {}
    for nw in worker_counts:
        if isinstance(dataset, str):
            ld = NativeStoreLoader(dataset, batch_size, seq_max_length, num_threads=max(1, nw), drop_last=False)
        else:
            ld = DataLoader(dataset, shuffle=True, num_workers=nw, batch_size=batch_size, pin_memory=torch.cuda.is_available(),
                            collate_fn=collate_triples)
        start = time.perf_counter()
        for _ in range(epochs):
            for i, _batch in enumerate(ld):
                if max_batches is not None and i + 1 >= max_batches:
                    break
        out[nw] = time.perf_counter() - start
        if hasattr(ld, "close"):
            ld.close()
        if verbose:
            print(f"Finish with:{out[nw]} second, num_workers={nw}")
    return out
