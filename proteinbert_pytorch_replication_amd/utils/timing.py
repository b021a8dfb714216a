"""Wall-clock and device timers (reference ``shared_utils/util.py:1203-1263``: ``TimeMeasure``,
``Profiler``), plus a HIP-event step timer for the training loops."""
from __future__ import annotations

import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, Optional


class TimeMeasure:
    """``with TimeMeasure('loading'):`` logs the start and the elapsed time."""

    def __init__(self, opening_statement: Optional[str] = None, logger=None):
        from .log import log
        self.opening_statement = opening_statement
        self.log = logger or log
        self.elapsed = 0.0

    def __enter__(self):
        self.start = time.perf_counter()
        if self.opening_statement:
            self.log(self.opening_statement)
        return self

    def __exit__(self, *exc):
        self.elapsed = time.perf_counter() - self.start
        if self.opening_statement:
            self.log("Finished after %.3f seconds." % self.elapsed)
        return False


class Profiler:
    """Named accumulating sections: ``with prof.measure('fwd'): ...``; ``prof.report()``."""

    def __init__(self):
        self.totals: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)

    @contextmanager
    def measure(self, name: str):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.totals[name] += time.perf_counter() - t0
            self.counts[name] += 1

    def report(self) -> str:
        lines = ["%-24s %10.4f s  %6d calls" % (k, v, self.counts[k])
                 for k, v in sorted(self.totals.items(), key=lambda kv: -kv[1])]
        return "\n".join(lines)


class DummyContext:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


class StepTimer:
    """Device-side step timing with HIP events (no host sync until :meth:`elapsed_ms`)."""

    def __init__(self, device=None):
        import torch
        self.cuda = torch.cuda.is_available() and (device is None or str(device).startswith("cuda"))
        self._t0 = None

    def start(self) -> None:
        import torch
        if self.cuda:
            self._e0 = torch.cuda.Event(enable_timing=True)
            self._e1 = torch.cuda.Event(enable_timing=True)
            self._e0.record()
        else:
            self._t0 = time.perf_counter()

    def stop(self) -> None:
        if self.cuda:
            self._e1.record()
        else:
            self._t1 = time.perf_counter()

    def elapsed_ms(self) -> float:
        if self.cuda:
            self._e1.synchronize()
            return self._e0.elapsed_time(self._e1)
        return (self._t1 - self._t0) * 1000.0
