"""Host (CPU) time per piece of the eager training step, including the autograd worker thread's Python
backward functions (which cProfile on the main thread does not see): every custom autograd Function's
forward / backward, the fused heads and the optimizer calls are wrapped with perf_counter accumulators.

    python tools/host_breakdown.py [--steps 20]
"""
import argparse
import collections
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO  # noqa: E402
from proteinbert_pytorch_replication_amd.models import ProteinBERT  # noqa: E402
from proteinbert_pytorch_replication_amd.ops import global_track, local_track  # noqa: E402
from proteinbert_pytorch_replication_amd.train.optim import FusedAdam  # noqa: E402
from proteinbert_pytorch_replication_amd.train.step import PretrainStep  # noqa: E402

measuring = {"on": False}
acc = collections.defaultdict(float)
cnt = collections.Counter()
PROF = os.environ.get("PBX_HB_PROFILE") == "1"   # cProfile inside the wrapped calls (autograd thread included)
if PROF:
    import cProfile
    import pstats
    _prof = cProfile.Profile()
_depth = {"n": 0}


def wrap(owner, name, label):
    fn = getattr(owner, name)
    # classes: the plain function behind a staticmethod; instances: the bound method itself
    raw = (fn.__func__ if hasattr(fn, "__func__") else fn) if isinstance(owner, type) else fn

    def timed(*a, **k):
        t = time.perf_counter()
        top = PROF and _depth["n"] == 0 and measuring["on"]
        if top:
            _prof.enable()
        _depth["n"] += 1
        try:
            return raw(*a, **k)
        finally:
            _depth["n"] -= 1
            if top:
                _prof.disable()
            acc[label] += time.perf_counter() - t
            cnt[label] += 1
    is_static = isinstance(owner, type) and isinstance(owner.__dict__.get(name), staticmethod)
    setattr(owner, name, staticmethod(timed) if is_static else timed)


for mod in (global_track, local_track):
    for n in dir(mod):
        c = getattr(mod, n)
        if isinstance(c, type) and issubclass(c, torch.autograd.Function) and c is not torch.autograd.Function:
            for m in ("forward", "backward"):
                if m in c.__dict__:
                    wrap(c, m, f"{n}.{m}")

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda")
torch.manual_seed(0)
m = ProteinBERT(sequences_length=512, num_annotations=8943, local_dim=128, global_dim=512, key_dim=64, num_heads=4,
                num_blocks=6, device=dev, backend="hip")
opt = FusedAdam(m.parameters(), lr=2e-4)
step = PretrainStep(m, opt)
wrap(opt, "zero_grad", "opt.zero_grad")
wrap(opt, "step", "opt.step")
wrap(opt, "set_nonfinite_skip", "opt.set_nonfinite_skip")
gen = SyntheticUniRefGO(512, 8943, 512, dev, seed=1)
for _ in range(5):
    step(*gen.next_batch())
torch.cuda.synchronize()
acc.clear()
cnt.clear()
measuring["on"] = True
t0 = time.perf_counter()
tb = 0.0
for _ in range(a.steps):
    t = time.perf_counter()
    X, Y, W = gen.next_batch()
    tb += time.perf_counter() - t
    step(X, Y, W)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
n = a.steps
print(f"issue {1e3 * (t1 - t0) / n:.3f} ms/step  complete {1e3 * (t2 - t0) / n:.3f} ms/step  batch {1e3 * tb / n:.3f}")
for k, v in sorted(acc.items(), key=lambda x: -x[1]):
    print(f"  {1e3 * v / n:7.3f} ms/step  {cnt[k] / n:5.1f} calls/step  {1e6 * v / max(1, cnt[k]):8.1f} us/call  {k}")
if PROF:
    pstats.Stats(_prof).sort_stats("tottime").print_stats(30)
