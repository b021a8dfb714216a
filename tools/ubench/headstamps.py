"""Phase timestamps (s_memtime) of the local-head kernel from an instrumented build of glob.hip
(tools/ubench/abl/libglob_st.so: ST() stamps by thread 0 of workgroups 0 and 300)."""
import ctypes

import torch

B, L, V, C = 512, 512, 26, 128
dev = torch.device("cuda")
_ = torch.cuda.is_available()
lib = ctypes.CDLL("tools/ubench/abl/libglob_st.so", mode=ctypes.RTLD_LOCAL)
P, I = ctypes.c_void_p, ctypes.c_int
lib.pbx_local_head.argtypes = [P, P, P, P, P, P, P, P, P, I, I, I, P]
lib.pbx_set_stamps.argtypes = [P]
h = (torch.randn(B, L, C, device=dev) * 0.5).to(torch.bfloat16)
wo = torch.randn(V, C, device=dev) * 0.1
bo = torch.zeros(V, device=dev)
y = torch.randint(0, V, (B, L), device=dev)
wl = torch.ones(B, L, device=dev)
dh = torch.empty_like(h)
dwo = torch.empty(L, V, C, device=dev)
dbo = torch.empty(L, V, device=dev)
loss = torch.zeros(2, device=dev)
stamps = torch.zeros(32, dtype=torch.int64, device=dev)
lib.pbx_set_stamps(ctypes.c_void_p(stamps.data_ptr()))
st = torch.cuda.current_stream().cuda_stream
for it in range(3):
    lib.pbx_local_head(h.data_ptr(), wo.data_ptr(), bo.data_ptr(), y.data_ptr(), wl.data_ptr(), dh.data_ptr(),
                       dwo.data_ptr(), dbo.data_ptr(), loss.data_ptr(), B, L, V, st)
torch.cuda.synchronize()
s = stamps.cpu().tolist()
names = ["start", "h loads issued", "logits", "softmax stats", "P norm", "CE", "dz", "dWo", "dbo", "dh", "end"]
for base in (0, 16):
    t = s[base:base + 11]
    print("WG", 0 if base == 0 else 300, " ".join(f"{names[i]}:{t[i] - t[i - 1]}" for i in range(1, 11)),
          "total", t[10] - t[0], flush=True)
