"""Per-kernel timing of the fused local-track kernels on the paper config (B=256, L=512).

    python tools/kbench.py [--B 256] [--L 512] [--iters 20]

Prints us/call and effective TFLOP/s (MFMA FLOPs the kernel performs) for each launcher, with
variants (tile sizes) where the launcher exposes them.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from proteinbert_pytorch_replication_amd.ops import _lib  # noqa: E402
from proteinbert_pytorch_replication_amd.ops import local_track as lt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=256)
ap.add_argument("--L", type=int, default=512)
ap.add_argument("--iters", type=int, default=20)
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


def report(name, us, flops=None, bytes_=None):
    extra = ""
    if flops:
        extra += f"  {flops / us / 1e6:8.1f} TFLOP/s"
    if bytes_:
        extra += f"  {bytes_ / us / 1e6:8.2f} TB/s"
    print(f"{name:40s} {us:9.1f} us{extra}", flush=True)


x = (torch.randn(B, L, C, device=dev) * 0.5).to(bf)
w = torch.randn(C, C, KS, device=dev) * 0.03
wpn, wtn = torch.empty(KS, C, C, dtype=bf, device=dev), torch.empty(KS, C, C, dtype=bf, device=dev)
_lib.call("pbx_pack_conv", w.data_ptr(), wpn.data_ptr(), wtn.data_ptr(), KS, st)
wpw, wtw = wpn, wtn
bias = torch.zeros(C, device=dev)
gb = torch.zeros(B, C, device=dev)
act = lambda: torch.empty_like(x)  # noqa: E731
pre_n, pre_w, s1 = act(), act(), act()
conv_flops = 2 * 2 * B * L * C * C * KS
for BM in (256, 128):
    T = (L + BM - 1) // BM
    stt = torch.empty(B, T, 2, device=dev)
    us = timeit(lambda: _lib.call("pbx_conv_fwd", x.data_ptr(), wpn.data_ptr(), wpw.data_ptr(), bias.data_ptr(),
                                  bias.data_ptr(), gb.data_ptr(), pre_n.data_ptr(), pre_w.data_ptr(), s1.data_ptr(),
                                  stt.data_ptr(), B, L, KS, dil, BM, st))
    report(f"conv_fwd BM={BM}", us, conv_flops, 4 * x.numel() * 2)
    dx, dpn, dpw = act(), act(), act()
    us = timeit(lambda: _lib.call("pbx_conv_dgrad", s1.data_ptr(), pre_n.data_ptr(), pre_w.data_ptr(),
                                  wtn.data_ptr(), wtw.data_ptr(), dx.data_ptr(), dpn.data_ptr(), dpw.data_ptr(), B, L,
                                  KS, dil, BM, st))
    report(f"conv_dgrad BM={BM}", us, conv_flops, 6 * x.numel() * 2)
# fragment-streamed forms (conv2.hip), checked against the v1 outputs of the same inputs
bias2 = torch.randn(C, device=dev) * 0.1
gb2 = torch.randn(B, C, device=dev) * 0.1
T1 = (L + 255) // 256
st_a = torch.empty(B, T1, 2, device=dev)
ref = [act() for _ in range(3)]
_lib.call("pbx_conv_fwd", x.data_ptr(), wpn.data_ptr(), wpw.data_ptr(), bias2.data_ptr(), bias2.data_ptr(),
          gb2.data_ptr(), ref[0].data_ptr(), ref[1].data_ptr(), ref[2].data_ptr(), st_a.data_ptr(), B, L, KS, dil, 256,
          st)
fpn, ftn_ = torch.empty_like(wpn), torch.empty_like(wpn)
_lib.call("pbx_pack_conv_frag", w.data_ptr(), fpn.data_ptr(), ftn_.data_ptr(), KS, st)
T2 = (L + 127) // 128
st_b = torch.empty(B, T2, 2, device=dev)
new = [act() for _ in range(3)]
for tbm in (128, 256):
    st_b = torch.empty(B, (L + tbm - 1) // tbm, 2, device=dev)
    fwd2 = lambda: _lib.call("pbx_conv_fwd3", x.data_ptr(), fpn.data_ptr(), fpn.data_ptr(), bias2.data_ptr(),  # noqa
                             bias2.data_ptr(), gb2.data_ptr(), new[0].data_ptr(), new[1].data_ptr(),
                             new[2].data_ptr(), st_b.data_ptr(), B, L, KS, dil, tbm, st)
    fwd2()
    torch.cuda.synchronize()
    for nm, u, v in zip(("pre_n", "pre_w", "s1"), ref, new):
        print(f"  fwd3/{tbm} vs fwd {nm}: max|diff| {float((u.float() - v.float()).abs().max()):.4g}  "
              f"max|ref| {float(u.float().abs().max()):.3g}", flush=True)
    report(f"conv_fwd3 tile {tbm} (frag-streamed W)", timeit(fwd2), conv_flops, 4 * x.numel() * 2)
dref = [act() for _ in range(3)]
dnew = [act() for _ in range(3)]
ds1 = (torch.randn(B, L, C, device=dev) * 0.1).to(bf)
_lib.call("pbx_conv_dgrad", ds1.data_ptr(), ref[0].data_ptr(), ref[1].data_ptr(), wtn.data_ptr(), wtw.data_ptr(),
          dref[0].data_ptr(), dref[1].data_ptr(), dref[2].data_ptr(), B, L, KS, dil, 256, st)
dg2 = lambda: _lib.call("pbx_conv_dgrad3", ds1.data_ptr(), ref[0].data_ptr(), ref[1].data_ptr(),  # noqa
                        ftn_.data_ptr(), ftn_.data_ptr(), dnew[0].data_ptr(), dnew[1].data_ptr(), dnew[2].data_ptr(),
                        B, L, KS, dil, st)
dg2()
torch.cuda.synchronize()
for nm, u, v in zip(("dx", "dpre_n", "dpre_w"), dref, dnew):
    print(f"  dgrad3 vs dgrad {nm}: max|diff| {float((u.float() - v.float()).abs().max()):.4g}  "
          f"max|ref| {float(u.float().abs().max()):.3g}", flush=True)
report("conv_dgrad3 (frag-streamed W)", timeit(dg2), conv_flops, 6 * x.numel() * 2)

dw0 = torch.zeros(C, C, KS, device=dev)
dw1 = torch.zeros(C, C, KS, device=dev)
db0 = torch.zeros(C, device=dev)
db1 = torch.zeros(C, device=dev)
for R in (32, 64, 128):
    slab = torch.empty(R, 2, KS, C, C, device=dev)
    bslab = torch.empty(R, 2, C, device=dev)
    us = timeit(lambda: _lib.call("pbx_wgrad", pre_n.data_ptr(), pre_w.data_ptr(), x.data_ptr(), slab.data_ptr(),
                                  bslab.data_ptr(), dw0.data_ptr(), dw1.data_ptr(), db0.data_ptr(), db1.data_ptr(), B,
                                  L, KS, dil, 2, R, 1, st))
    report(f"conv wgrad+reduce R={R}", us, conv_flops)

# LDS-DMA form (csrc/wgrad.hip), checked against the v1 result of the same inputs
pre_n.copy_((torch.randn(B, L, C, device=dev) * 0.5).to(bf))
pre_w.copy_((torch.randn(B, L, C, device=dev) * 0.5).to(bf))
ref = []
for R, fn in ((48, "pbx_wgrad"), (64, "pbx_wgrad2")):
    for t in (dw0, dw1, db0, db1):
        t.zero_()
    slab = torch.empty(R, 2, KS, C, C, device=dev)
    bslab = torch.empty(R, 2, C, device=dev)
    if fn == "pbx_wgrad":
        call = lambda: _lib.call(fn, pre_n.data_ptr(), pre_w.data_ptr(), x.data_ptr(), slab.data_ptr(),  # noqa: E731
                                 bslab.data_ptr(), dw0.data_ptr(), dw1.data_ptr(), db0.data_ptr(), db1.data_ptr(),
                                 B, L, KS, dil, 2, R, 1, st)
    else:
        call = lambda: _lib.call(fn, pre_n.data_ptr(), pre_w.data_ptr(), x.data_ptr(), slab.data_ptr(),  # noqa: E731
                                 bslab.data_ptr(), dw0.data_ptr(), dw1.data_ptr(), db0.data_ptr(), db1.data_ptr(),
                                 B, L, dil, 2, R, st)
    call()
    torch.cuda.synchronize()
    ref.append([t.clone() for t in (dw0, dw1, db0, db1)])
    report(f"{fn} R={R}", timeit(call), conv_flops)
for nm, u, v in zip(("dw_n", "dw_w", "db_n", "db_w"), ref[0], ref[1]):
    print(f"  wgrad2 vs wgrad {nm}: max|diff| {float((u - v).abs().max()):.4g}  max|ref| {float(u.abs().max()):.3g}",
          flush=True)
for R in (32, 128):
    slab = torch.empty(R, 2, KS, C, C, device=dev)
    bslab = torch.empty(R, 2, C, device=dev)
    report(f"pbx_wgrad2 R={R}", timeit(lambda: _lib.call(
        "pbx_wgrad2", pre_n.data_ptr(), pre_w.data_ptr(), x.data_ptr(), slab.data_ptr(), bslab.data_ptr(),
        dw0.data_ptr(), dw1.data_ptr(), db0.data_ptr(), db1.data_ptr(), B, L, dil, 2, R, st)), conv_flops)
