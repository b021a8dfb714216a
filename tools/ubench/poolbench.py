"""Standalone timing of the B=512, L=512 attention-pool v2 kernels and the LN/MLP kernels
(event-timed, mean of --iters launches).  PBX_HIP_LIB selects an ablation build.
    python tools/ubench/poolbench.py [--B 512] [--L 512]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from proteinbert_pytorch_replication_amd.ops import _lib  # noqa: E402
from proteinbert_pytorch_replication_amd.ops import local_track as lt  # noqa: E402,F401

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=512)
ap.add_argument("--L", type=int, default=512)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
B, L, C, NJ = a.B, a.L, 128, 512
dev = torch.device("cuda")
st = _lib.stream_ptr(dev)
bf = torch.bfloat16


def timeit(fn, n=a.iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000.0


P = lambda t: t.data_ptr()  # noqa: E731
x = torch.randn(B, L, C, device=dev).to(bf)
T1 = (L + 127) // 128
st1 = torch.zeros(B, T1, 2, device=dev)
st1[..., 1] = 128 * C
g1 = torch.ones(L, C, device=dev)
be1 = torch.zeros(L, C, device=dev)
wl = (torch.randn(C, C, device=dev) * 0.08).to(bf)
bl = torch.zeros(C, device=dev)
pre_l, s2 = torch.empty_like(x), torch.empty_like(x)
T2 = (L + 31) // 32
st2 = torch.empty(B, T2, 2, device=dev)
for store in (True, False):
    us = timeit(lambda: _lib.call("pbx_ln_linear_fwd", P(x), P(st1), T1, 128, P(g1), P(be1), P(wl), P(bl),
                                  P(pre_l) if store else None, P(s2), P(st2), B, L, 1e-5, st))
    print(f"ln_linear_fwd store_pre={store}: {us:8.1f} us", flush=True)
g2 = torch.ones(L, C, device=dev)
be2 = torch.zeros(L, C, device=dev)
wv = (torch.randn(NJ, C, device=dev) * 0.05).to(bf)
h2 = torch.empty_like(x)
TV = (L + 63) // 64
vpart = torch.empty(B, TV * (2 if lt.ATTN_FWD2_CFG & 15 == 12 else 1), NJ, device=dev)   # 12: rows per 32 positions
gfrag = torch.empty(B, 2 * TV, NJ * 32, device=dev, dtype=bf)
us = timeit(lambda: _lib.call("pbx_ln_attn_fwd2", P(s2), P(st2), P(g2), P(be2), P(wv), P(h2), P(vpart), P(gfrag),
                              B, L, NJ, lt.ATTN_FWD2_CFG, 1e-5, st))
print(f"ln_attn_fwd2: {us:8.1f} us", flush=True)
dv = torch.randn(B, NJ, device=dev) * 1e-3
dh2 = torch.empty_like(x)
sums2 = torch.empty(B, T2, 2, device=dev)
us = timeit(lambda: _lib.call("pbx_attn_bwd2", P(gfrag), P(s2), P(st2), P(g2), None, P(dv), (L + 31) // 32 * 32,
                              P(wv), P(dh2), P(sums2), B, L, NJ, 1e-5, st))
print(f"attn_bwd2: {us:8.1f} us", flush=True)
dh1 = torch.empty_like(x)
TS1 = (L + 1) // 2
sums1 = torch.empty(B, TS1, 2, device=dev)
consts = torch.empty(B, 8, device=dev)
dgb = torch.empty(B, C, device=dev)
acc = [torch.zeros(L, C, device=dev) for _ in range(4)]
dwl, dbl = torch.zeros(C, C, device=dev), torch.zeros(C, device=dev)
for recomp in (False, True):
    for wgcu in (0, 2):
        us = timeit(lambda: _lib.call("pbx_ln2_linear_bwd2", P(dh2), P(s2), P(st2), P(sums2), T2, P(g2),
                                      None if recomp else P(pre_l), P(bl) if recomp else None, P(x), P(st1), T1,
                                      128, P(g1), P(be1), P(wl), P(consts), P(dh1), P(sums1), *[P(t) for t in acc],
                                      P(dwl), P(dbl), P(dgb), None, None, B, L, 1e-5, wgcu, None, 0, st))
        print(f"ln2_linear_bwd recompute={recomp} wg/cu={wgcu}: {us:8.1f} us", flush=True)
ds1 = torch.empty_like(x)
us = timeit(lambda: _lib.call("pbx_ln1_finalize", P(dh1), P(x), P(st1), T1, 128, P(sums1), TS1, P(g1), P(ds1),
                              P(dgb), B, L, 1e-5, st))
print(f"ln1_finalize: {us:8.1f} us", flush=True)
