"""Chunking / task-splitting helpers (reference ``shared_utils/util.py:236-369``)."""
from __future__ import annotations

from itertools import islice
from typing import Iterable, Iterator, List, Tuple


def to_chunks(iterable: Iterable, chunk_size: int) -> Iterator[List]:
    """Yield consecutive lists of ``chunk_size`` items (the last may be shorter)."""
    if chunk_size <= 0:
        raise ValueError("chunk_size must be positive")
    it = iter(iterable)
    while True:
        chunk = list(islice(it, chunk_size))
        if not chunk:
            return
        yield chunk


def get_chunk_slice(size: int, n_chunks: int, chunk_index: int) -> Tuple[int, int]:
    """[start, end) of chunk ``chunk_index`` when ``size`` items are split into ``n_chunks``."""
    if not 0 <= chunk_index < n_chunks:
        raise ValueError("chunk_index out of range")
    base, rem = divmod(size, n_chunks)
    start = chunk_index * base + min(chunk_index, rem)
    return start, start + base + (1 if chunk_index < rem else 0)


def get_chunk_intervals(size: int, chunk_size: int) -> List[Tuple[int, int]]:
    return [(s, min(s + chunk_size, size)) for s in range(0, size, chunk_size)]


def get_job_and_subjob_indices(n_jobs: int, n_tasks: int, task_index: int) -> Tuple[int, int, int]:
    """Map a flat task index onto (job, subjob, n_subjobs) when n_tasks >= n_jobs tasks share jobs."""
    n_tasks_per_job = n_tasks // n_jobs
    extra = n_tasks % n_jobs
    job = 0
    start = 0
    while True:
        n = n_tasks_per_job + (1 if job < extra else 0)
        if task_index < start + n:
            return job, task_index - start, n
        start += n
        job += 1
