"""Per-item phase timestamps (s_memtime, wave 0 of workgroup 0) of attn_bwd from an instrumented
build of ln.hip (tools/ubench/abl/libln_st.so), plus the kernel time, at the paper config B=512."""
import ctypes

import torch

B, L, C, NJ = 512, 512, 128, 512
dev = torch.device("cuda")
_ = torch.cuda.is_available()
import sys
lib = ctypes.CDLL(sys.argv[1] if len(sys.argv) > 1 else "tools/ubench/abl/libln_st.so", mode=ctypes.RTLD_LOCAL)
P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
lib.pbx_attn_bwd.argtypes = [P, P, P, P, P, P, I, P, P, P, I, I, I, I, F, P]
lib.pbx_set_stamps.argtypes = [P]
bf = torch.bfloat16
h2 = (torch.randn(B, L, C, device=dev) * 0.5).to(bf)
s2 = (torch.randn(B, L, C, device=dev) * 0.5).to(bf)
st2 = torch.zeros(B, 16, 2, device=dev)
st2[:, :, 1] = 32 * 128 * 0.25
g2 = torch.ones(L, C, device=dev)
dh2_in = (torch.randn(B, L, C, device=dev) * 0.01).to(bf)
dvpart = torch.randn(B, NJ, device=dev) * 0.01
wv = (torch.randn(NJ, C, device=dev) * 0.1).to(bf)
dh2 = torch.empty_like(h2)
sums2 = torch.empty(B, L // 32, 2, device=dev)
stamps = torch.zeros(64, dtype=torch.int64, device=dev)
lib.pbx_set_stamps(ctypes.c_void_p(stamps.data_ptr()))
stream = torch.cuda.current_stream().cuda_stream


def call():
    return lib.pbx_attn_bwd(h2.data_ptr(), s2.data_ptr(), st2.data_ptr(), g2.data_ptr(), dh2_in.data_ptr(),
                            dvpart.data_ptr(), 512, wv.data_ptr(), dh2.data_ptr(), sums2.data_ptr(), B, L, NJ, 8,
                            1e-5, stream)


call()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    call()
e1.record()
torch.cuda.synchronize()
print(f"attn_bwd {e0.elapsed_time(e1) / 10 * 1000:.1f} us", flush=True)
s = [x for x in stamps.cpu().tolist() if x]
d = [s[i] - s[i - 1] for i in range(1, len(s))]
print("deltas (prologue, then per item: load rows / jt loop / epilogue):", d, flush=True)
