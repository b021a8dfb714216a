"""Time the conv kernels (conv_fwd3 / conv_fwd5, csrc/conv2.hip / conv5.hip; conv_dgrad4,
csrc/conv4.hip; wgrad2, csrc/wgrad.hip)
at the bench shape through their exported launchers (whole sequences: no context-parallel halo rows), with
whatever library PBX_HIP_LIB names (a variant built by tools/ubench/build_flags.sh).

    python tools/ubench/convbench.py [--B 1024 --L 512]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from proteinbert_pytorch_replication_amd.ops import _lib, local_track  # noqa: E402,F401  (registers the launchers)

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=1024)
ap.add_argument("--L", type=int, default=512)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--tag", default="")
a = ap.parse_args()
B, L, C, KS, dil = a.B, a.L, 128, 9, 5
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


flops = 2 * 2 * B * L * C * C * KS
x = (torch.randn(B, L, C, device=dev) * 0.5).to(bf)
w = torch.randn(C, C, KS, device=dev) * 0.03
fp, ft = torch.empty(KS, C, C, dtype=bf, device=dev), torch.empty(KS, C, C, dtype=bf, device=dev)
_lib.call("pbx_pack_conv_frag", w.data_ptr(), fp.data_ptr(), ft.data_ptr(), KS, st)
bias = torch.randn(C, device=dev) * 0.1
gb = torch.randn(B, C, device=dev) * 0.1
pre_n, pre_w, s1 = (torch.empty_like(x) for _ in range(3))
stt = torch.empty(B, (L + 127) // 128, 2, device=dev)
fwd = lambda: _lib.call("pbx_conv_fwd3x", x.data_ptr(), fp.data_ptr(), fp.data_ptr(), bias.data_ptr(),  # noqa: E731
                        bias.data_ptr(), gb.data_ptr(), pre_n.data_ptr(), pre_w.data_ptr(), s1.data_ptr(),
                        stt.data_ptr(), B, L, KS, dil, 0, 0, st)
us = timeit(fwd)
print(f"[{a.tag}] conv_fwd3   {us:8.1f} us  {flops / us / 1e6:7.1f} TFLOP/s", flush=True)
fwd5 = lambda: _lib.call("pbx_conv_fwd5x", x.data_ptr(), fp.data_ptr(), fp.data_ptr(), bias.data_ptr(),  # noqa: E731
                         bias.data_ptr(), gb.data_ptr(), pre_n.data_ptr(), pre_w.data_ptr(), s1.data_ptr(),
                         stt.data_ptr(), B, L, KS, dil, 0, 0, st)
us = timeit(fwd5)
print(f"[{a.tag}] conv_fwd5   {us:8.1f} us  {flops / us / 1e6:7.1f} TFLOP/s", flush=True)
ds1 = (torch.randn(B, L, C, device=dev) * 0.1).to(bf)
dx, dpn, dpw = (torch.empty_like(x) for _ in range(3))
dg4 = lambda: _lib.call("pbx_conv_dgrad4x", ds1.data_ptr(), pre_n.data_ptr(), pre_w.data_ptr(), ft.data_ptr(),  # noqa
                        ft.data_ptr(), dx.data_ptr(), dpn.data_ptr(), dpw.data_ptr(), B, L, KS, dil, 0, 0, st)
us = timeit(dg4)
print(f"[{a.tag}] conv_dgrad4 {us:8.1f} us  {flops / us / 1e6:7.1f} TFLOP/s", flush=True)
# the FIN form (LN1 backward finalize fused in)
dh1 = (torch.randn(B, L, C, device=dev) * 0.1).to(bf)
g1 = torch.randn(L, C, device=dev) * 0.1 + 1.0
T1 = (L + 127) // 128
st1 = torch.stack([torch.zeros(B, T1, device=dev), torch.full((B, T1), 128.0 * C * 0.25, device=dev)], -1)
sums1 = torch.randn(B, 4, 2, device=dev)
dgb = torch.zeros(B, C, device=dev)
fin_args = lambda: [dh1.data_ptr(), s1.data_ptr(), st1.data_ptr(), T1, 128, sums1.data_ptr(), 4, g1.data_ptr(),  # noqa
                    pre_n.data_ptr(), pre_w.data_ptr(), ft.data_ptr(), ft.data_ptr(), dx.data_ptr(), dpn.data_ptr(),
                    dpw.data_ptr(), dgb.data_ptr()]
us = timeit(lambda: _lib.call("pbx_conv_dgrad4f", *fin_args(), B, L, KS, dil, 1e-5, st))
print(f"[{a.tag}] conv_dgrad4<FIN> {us:8.1f} us  {flops / us / 1e6:7.1f} TFLOP/s", flush=True)
slab = torch.empty(64 * 2 * KS * C * C, device=dev)
bslab = torch.empty(64 * 2 * C, device=dev)
dwn, dww = torch.zeros(C, C, KS, device=dev), torch.zeros(C, C, KS, device=dev)
dbn, dbw = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
for R in (56, 64):
    wg = lambda: _lib.call("pbx_wgrad2", dpn.data_ptr(), dpw.data_ptr(), x.data_ptr(), slab.data_ptr(),  # noqa
                           bslab.data_ptr(), dwn.data_ptr(), dww.data_ptr(), dbn.data_ptr(), dbw.data_ptr(), B, L, dil,
                           2, R, st)
    us = timeit(wg)
    print(f"[{a.tag}] wgrad2 R={R} {us:8.1f} us  {flops / us / 1e6:7.1f} TFLOP/s (incl. slab fold)", flush=True)
