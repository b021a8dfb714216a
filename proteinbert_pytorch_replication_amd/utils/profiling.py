"""On-demand tracing of training steps.

The reference only times iterations on the host (``ProteinBERT/utils.py:284,306,312``).  Here:

* :class:`StepProfiler` - a ``torch.profiler`` window over training steps ``[start, start + count)``
  (HIP kernels through roctracer on ROCm, CPU ops elsewhere), written as a Chrome trace plus a
  per-kernel table; kernel-level counters come from ``rocprofv3`` around the same command
  (``tools/gpu_prof.sh``, ``tools/gpu_pmc_final.sh``).
* :func:`marker` - a named range (``torch.cuda.nvtx`` -> roctx on ROCm) that shows up in rocprofv3
  / the trace, around phases such as ``pbx/step`` or ``pbx/checkpoint``.
"""
from __future__ import annotations

import os
from contextlib import contextmanager
from typing import Optional

import torch


@contextmanager
def marker(name: str):
    """roctx range on a GPU build (visible in ``rocprofv3 --marker-trace`` and torch traces)."""
    use = torch.cuda.is_available()
    if use:
        torch.cuda.nvtx.range_push(name)
    try:
        with torch.profiler.record_function(name):
            yield
    finally:
        if use:
            torch.cuda.nvtx.range_pop()


class StepProfiler:
    """Profile steps ``[start, start + count)`` (1-based step counter as in :func:`..train.pretrain`)."""

    def __init__(self, out_dir: str, start: int, count: int = 1, rank: int = 0):
        self.out_dir, self.start, self.count, self.rank = out_dir, int(start), int(count), rank
        self.prof: Optional[torch.profiler.profile] = None
        self.trace_path: Optional[str] = None

    @classmethod
    def from_spec(cls, spec: Optional[str], out_dir: Optional[str], rank: int = 0) -> Optional["StepProfiler"]:
        """``spec`` = ``START[:COUNT]`` (e.g. ``"20:3"``) or None."""
        if not spec:
            return None
        s, _, c = str(spec).partition(":")
        return cls(out_dir or ".", int(s), int(c or 1), rank)

    def before_step(self, step: int) -> None:
        if step == self.start and self.prof is None:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self.prof = torch.profiler.profile(activities=acts, record_shapes=False)
            self.prof.__enter__()

    def after_step(self, step: int) -> None:
        if self.prof is not None and step >= self.start + self.count - 1:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            self.prof.__exit__(None, None, None)
            os.makedirs(self.out_dir, exist_ok=True)
            self.trace_path = os.path.join(self.out_dir, f"pbx_trace_rank{self.rank}_steps{self.start}-"
                                                         f"{self.start + self.count - 1}.json")
            self.prof.export_chrome_trace(self.trace_path)
            key = "self_cuda_time_total" if torch.cuda.is_available() else "self_cpu_time_total"
            with open(self.trace_path.replace(".json", ".txt"), "w") as f:
                f.write(self.prof.key_averages().table(sort_by=key, row_limit=40))
            self.prof = None
