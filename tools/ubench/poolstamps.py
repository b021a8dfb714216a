"""Per-phase clocks (s_memtime, lane 0 of waves 0-7 of workgroups 0-3) of the attention-pool forward
ln_attn_fwd2 from the instrumented build (tools/ubench/build_flags.sh st -DPBX_STAMPS), B=512 L=512.
    python tools/ubench/poolstamps.py [lib]"""
import ctypes
import sys

import torch

B, L, C, NJ = 512, 512, 128, 512
dev = torch.device("cuda")
_ = torch.cuda.is_available()
lib = ctypes.CDLL(sys.argv[1] if len(sys.argv) > 1 else "tools/ubench/abl/libpbx_st.so", mode=ctypes.RTLD_LOCAL)
P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
lib.pbx_ln_attn_fwd2.argtypes = [P, P, P, P, P, P, P, P, I, I, I, F, I, P]
PRE = int(sys.argv[2]) if len(sys.argv) > 2 else 0
lib.pbx_set_stamps.argtypes = [P]
bf = torch.bfloat16
s2 = (torch.randn(B, L, C, device=dev) * 0.5).to(bf)
st2 = torch.zeros(B, L // 32, 2, device=dev)
st2[:, :, 1] = 32 * 128 * 0.25
g2 = torch.ones(L, C, device=dev)
be2 = torch.zeros(L, C, device=dev)
wv = (torch.randn(NJ, C, device=dev) * 0.1).to(bf)
h2 = torch.empty(B, L, C, device=dev, dtype=bf)
TV = (L + 63) // 64
vpart = torch.empty(B, TV, NJ, device=dev)
gfrag = torch.empty(B, 2 * TV, NJ * 32, device=dev, dtype=bf)
stamps = torch.zeros(4 * 8 * 64, dtype=torch.int64, device=dev)
assert lib.pbx_set_stamps(ctypes.c_void_p(stamps.data_ptr())) == 0
stream = torch.cuda.current_stream().cuda_stream


def run():
    r = lib.pbx_ln_attn_fwd2(s2.data_ptr(), st2.data_ptr(), g2.data_ptr(), be2.data_ptr(), wv.data_ptr(),
                             h2.data_ptr(), vpart.data_ptr(), gfrag.data_ptr(), B, L, NJ, 1e-5, PRE, stream)
    assert r == 0, r


for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    run()
e1.record()
torch.cuda.synchronize()
print(f"kernel {e0.elapsed_time(e1) * 100:.1f} us (mean of 10)")
stamps.zero_()
run()
torch.cuda.synchronize()
s = stamps.view(32, 64).cpu()
t0 = s[:, 0][s[:, 0] > 0].min().item()
names = ["start", "staged"] + [f"it{i}_{n}" for i in range(2) for n in
                               (["begin", "stats", "frags"] + [f"jt{j}" for j in range(16)] + ["end"])]
print("clock cycles since the earliest wave start; mean / min / max over 32 waves (4 WGs x 8)")
for k, n in enumerate(names):
    col = s[:, k]
    ok = col > 0
    if ok.sum() == 0:
        continue
    v = (col[ok] - t0).double()
    print(f"{n:12s} {v.mean().item():9.0f} {v.min().item():9.0f} {v.max().item():9.0f}")
