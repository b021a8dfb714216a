"""conv_dgrad4<FIN> (csrc/conv4.hip, three phases per tile) vs conv_dgrad5 (csrc/conv5.hip, persistent,
next tile's prologue inside the MFMA loop): outputs compared, then timed.  B = 1024, L = 512 by default.
    python tools/ubench/dgrad5bench.py [--B 1024 --L 512]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from proteinbert_pytorch_replication_amd.ops import _lib, local_track as lt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=1024)
ap.add_argument("--L", type=int, default=512)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--timing-only", action="store_true", help="exit 0 on mismatch (ablation builds)")
a = ap.parse_args()
B, L, C, KS, dil = a.B, a.L, 128, 9, 5
dev = torch.device("cuda")
st = _lib.stream_ptr(dev)
torch.manual_seed(0)
bf = torch.bfloat16
T1 = (L + lt.BM1 - 1) // lt.BM1
TS1 = (L + 1) // 2
dh1, s1, gdn, gdw = ((torch.randn(B, L, C, device=dev) * 0.5).to(bf) for _ in range(4))
st1 = torch.zeros(B, T1, 2, device=dev)
st1[..., 0] = torch.randn(B, T1, device=dev) * 0.1
st1[..., 1] = lt.BM1 * C * 0.25
sums1 = torch.randn(B, TS1, 2, device=dev) * 0.01
g1 = torch.randn(L, C, device=dev) * 0.2 + 1
wn, ww = torch.randn(C, C, KS, device=dev) * 0.03, torch.randn(C, C, KS, device=dev) * 0.03
_, wtn = lt.pack_conv(wn)
_, wtw = lt.pack_conv(ww)


lnc = torch.empty(B, 4, device=dev)


def run(name):
    extra = (lnc.data_ptr(),) if name == "pbx_conv_dgrad5f" else ()
    dx, dpn, dpw = (torch.full_like(dh1, 7.0) for _ in range(3))
    dgb = torch.zeros(B, C, device=dev)
    fn = lambda: _lib.call(name, dh1.data_ptr(), s1.data_ptr(), st1.data_ptr(), T1, lt.BM1,  # noqa: E731
                           sums1.data_ptr(), TS1, g1.data_ptr(), gdn.data_ptr(), gdw.data_ptr(), wtn.data_ptr(),
                           wtw.data_ptr(), dx.data_ptr(), dpn.data_ptr(), dpw.data_ptr(), dgb.data_ptr(), *extra, B, L,
                           KS, dil, 1e-5, st)
    fn()
    torch.cuda.synchronize()
    outs = [dx.clone(), dpn.clone(), dpw.clone(), dgb.clone()]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return outs, e0.elapsed_time(e1) / a.iters * 1000.0


o4, t4 = run("pbx_conv_dgrad4f")
o5, t5 = run("pbx_conv_dgrad5f")
ok = True
for n, x4, x5 in zip(["dx", "dpn", "dpw", "dgb"], o4, o5):
    d = (x4.float() - x5.float()).abs().max().item()
    ref = x4.float().abs().max().item()
    print(f"{n}: max |diff| {d:.3e} (max |ref| {ref:.3e})")
    ok = ok and d <= 1e-3 * ref
print(f"B={B} L={L}: conv_dgrad4<FIN> {t4:.1f} us   conv_dgrad5 {t5:.1f} us   match={ok}", flush=True)
if not ok:   # where do they differ: per (sample, 128-row tile) and per row within the tile
    bad = ((o4[1].float() - o5[1].float()).abs().amax(dim=2) > 1e-2)          # [B, L]
    T = (L + 127) // 128
    bt = bad.view(B, T, 128).any(dim=2)
    print("bad tiles:", int(bt.sum()), "of", B * T, " first:", bt.nonzero()[:8].tolist())
    print("bad rows within tiles (histogram of row % 128, first 16 rows / last 16):",
          bad.view(B, T, 128).sum(dim=(0, 1))[:16].tolist(), bad.view(B, T, 128).sum(dim=(0, 1))[-16:].tolist())
    badc = ((o4[1].float() - o5[1].float()).abs() > 1e-2).view(-1, 128).sum(dim=0)
    print("bad channels:", badc.tolist()[:32])
sys.exit(0 if ok or a.timing_only else 1)
