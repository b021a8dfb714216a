"""Time pbx_ln_attn_fwd from an ablation build of ln.hip (tools/ubench/abl/libln_abl<N>.so)."""
import ctypes
import sys

import torch

B, L, C, NJ = 512, 512, 128, 512
dev = torch.device("cuda")
_ = torch.cuda.is_available()
P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
s2 = (torch.randn(B, L, C, device=dev) * 0.5).to(torch.bfloat16)
st2 = torch.zeros(B, 16, 2, device=dev)
st2[:, :, 1] = 32 * 128 * 0.25
g2 = torch.ones(L, C, device=dev)
be2 = torch.zeros(L, C, device=dev)
wv = (torch.randn(NJ, C, device=dev) * 0.1).to(torch.bfloat16)
h2 = torch.empty_like(s2)
vpart = torch.empty(B, L // 64, NJ, device=dev)
stream = torch.cuda.current_stream().cuda_stream
for path in sys.argv[1:]:
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    fn = lib.pbx_ln_attn_fwd
    fn.argtypes = [P, P, P, P, P, P, P, I, I, I, I, F, P]
    call = lambda: fn(s2.data_ptr(), st2.data_ptr(), g2.data_ptr(), be2.data_ptr(), wv.data_ptr(), h2.data_ptr(),  # noqa
                      vpart.data_ptr(), B, L, NJ, 8, 1e-5, stream)
    call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        call()
    e1.record()
    torch.cuda.synchronize()
    print(f"{path}: {e0.elapsed_time(e1) / 20 * 1000:.1f} us", flush=True)
