"""Recompute-form attention pool (csrc/pool.hip): numerics vs an fp32 torch oracle and kernel timing.
(Round 5 replaced the stored-GELU' pair: ln2_apply + ln_attn_fwd2 ~300 us and attn_bwd4 ~230 us at
B = 1024, L = 512 on the same box as pool_fwd 205 us / pool_bwd 291 us.)
    python tools/ubench/poolbench.py [--B 1024] [--L 512] [--check-only]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from proteinbert_pytorch_replication_amd.ops import _lib  # noqa: E402
from proteinbert_pytorch_replication_amd.ops import local_track  # noqa: E402,F401  (registers launchers)

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=1024)
ap.add_argument("--L", type=int, default=512)
ap.add_argument("--NJ", type=int, default=512)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--check-only", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda")
st = _lib.stream_ptr(dev)
bf = torch.bfloat16
C, NJ = 128, a.NJ


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


def stats(s2f, L):
    B = s2f.shape[0]
    T2 = (L + 31) // 32
    st2 = torch.empty(B, T2, 2, device=dev)
    for t in range(T2):
        x = s2f[:, 32 * t:min(L, 32 * t + 32)].reshape(B, -1)
        m = x.mean(1)
        st2[:, t, 0] = m
        st2[:, t, 1] = ((x - m[:, None]) ** 2).sum(1)
    return st2


def gelu_d(z):
    return 0.5 * (1 + torch.erf(z / 2 ** 0.5)) + z * torch.exp(-0.5 * z * z) / (2 * torch.pi) ** 0.5


def check(B, L):
    torch.manual_seed(0)
    TW = (L + 31) // 32
    s2 = (torch.randn(B, L, C, device=dev) * 2 + 0.3).to(bf)
    st2 = stats(s2.float(), L)
    g2 = torch.randn(L, C, device=dev) * 0.3 + 1
    be2 = torch.randn(L, C, device=dev) * 0.2
    wv = (torch.randn(NJ, C, device=dev) * 0.1).to(bf)
    h2 = torch.empty_like(s2)
    vpart = torch.empty(B, TW, NJ, device=dev)
    _lib.call("pbx_pool_fwd", s2.data_ptr(), st2.data_ptr(), g2.data_ptr(), be2.data_ptr(), wv.data_ptr(),
              h2.data_ptr(), vpart.data_ptr(), B, L, NJ, 1e-5, st)
    x = s2.float()
    m = x.mean((1, 2), keepdim=True)
    v = ((x - m) ** 2).mean((1, 2), keepdim=True)
    h2r = (x - m) / torch.sqrt(v + 1e-5) * g2 + be2
    e_h = (h2.float() - h2r).abs().max().item()
    z = h2.float() @ wv.float().t()                               # [B, L, NJ] from the kernel's bf16 h2
    gz = torch.nn.functional.gelu(z)
    pad = TW * 32 - L
    vr = torch.nn.functional.pad(gz, (0, 0, 0, pad)).view(B, TW, 32, NJ).sum(2)
    e_v = ((vpart - vr).abs().max() / vr.abs().max()).item()
    # backward
    dh2_in = (torch.randn(B, L, C, device=dev) * 0.5).to(bf)
    dv = torch.randn(B, NJ, device=dev) * 0.1
    dh2 = torch.empty_like(s2)
    sums2 = torch.empty(B, TW, 2, device=dev)
    _lib.call("pbx_pool_bwd", h2.data_ptr(), g2.data_ptr(), be2.data_ptr(), dh2_in.data_ptr(), dv.data_ptr(), 1,
              wv.data_ptr(), dh2.data_ptr(), sums2.data_ptr(), B, L, NJ, st)
    u = gelu_d(z) * dv[:, None, :]
    dr = dh2_in.float() + u @ wv.float()
    e_d = ((dh2.float() - dr).abs().max() / dr.abs().max()).item()
    dxh = dr * g2
    sa = torch.nn.functional.pad(dxh, (0, 0, 0, pad)).view(B, TW, 32, C).sum((2, 3))
    sc = torch.nn.functional.pad(dr * (h2.float() - be2), (0, 0, 0, pad)).view(B, TW, 32, C).sum((2, 3))
    e_sa = ((sums2[..., 0] - sa).abs().max() / sa.abs().max()).item()
    e_sc = ((sums2[..., 1] - sc).abs().max() / sc.abs().max()).item()
    print(f"check B={B} L={L}: h2 max|err| {e_h:.3e}  vpart rel {e_v:.3e}  dh2 rel {e_d:.3e}  "
          f"sums rel {e_sa:.3e} {e_sc:.3e}", flush=True)
    ok = e_h < 0.05 and e_v < 2e-3 and e_d < 1e-2 and e_sa < 1e-2 and e_sc < 1e-2
    return ok


ok = all([check(2, 500), check(3, 64), check(5, 77)])
print("numerics", "OK" if ok else "FAIL", flush=True)
if a.check_only:
    sys.exit(0 if ok else 1)

B, L = a.B, a.L
TW = (L + 31) // 32
s2 = torch.randn(B, L, C, device=dev).to(bf)
st2 = torch.zeros(B, TW, 2, device=dev)
st2[..., 1] = 32 * C
g2 = torch.ones(L, C, device=dev)
be2 = torch.zeros(L, C, device=dev)
wv = (torch.randn(NJ, C, device=dev) * 0.1).to(bf)
h2 = torch.empty_like(s2)
vpart = torch.empty(B, TW, NJ, device=dev)
dh2_in = torch.randn(B, L, C, device=dev).to(bf)
dv = torch.randn(B, NJ, device=dev) * 1e-2
dh2 = torch.empty_like(s2)
sums2 = torch.empty(B, TW, 2, device=dev)
mb = B * L * C * 2 / 1e6
us_f = timeit(lambda: _lib.call("pbx_pool_fwd", s2.data_ptr(), st2.data_ptr(), g2.data_ptr(), be2.data_ptr(),
                                wv.data_ptr(), h2.data_ptr(), vpart.data_ptr(), B, L, NJ, 1e-5, st))
us_b = timeit(lambda: _lib.call("pbx_pool_bwd", h2.data_ptr(), g2.data_ptr(), be2.data_ptr(), dh2_in.data_ptr(),
                                dv.data_ptr(), 1, wv.data_ptr(), dh2.data_ptr(), sums2.data_ptr(), B, L, NJ, st))
print(f"B={B} L={L}: pool_fwd {us_f:8.1f} us ({2 * mb / us_f:.2f} TB/s)   pool_bwd {us_b:8.1f} us "
      f"({3 * mb / us_b:.2f} TB/s)", flush=True)
