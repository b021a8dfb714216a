"""Fine-tune token head GEMM formulations: [B*L, 128] x [128, K] (K = 8), forward + weight grad."""
import torch
import torch.nn.functional as F
dev = "cuda"
M, C, K = 512 * 512, 128, 8
h = torch.randn(M, C, device=dev).to(torch.bfloat16)
W = torch.randn(K, C, device=dev) * 0.1
b = torch.zeros(K, device=dev)
g = torch.randn(M, K, device=dev)


def t(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000


print("fp32 F.linear (current)   %.1f us" % t(lambda: F.linear(h.float(), W, b)))
Wb = W.to(torch.bfloat16)
print("bf16 F.linear             %.1f us" % t(lambda: F.linear(h, Wb, b.to(torch.bfloat16))))
print("bf16 (W @ h^T)^T          %.1f us" % t(lambda: (Wb @ h.t()).t()))
print("bf16 mm h @ W^T           %.1f us" % t(lambda: torch.mm(h, Wb.t())))
Wp = torch.zeros(16, C, device=dev, dtype=torch.bfloat16)
Wp[:K] = Wb
print("bf16 mm padded K=16       %.1f us" % t(lambda: torch.mm(h, Wp.t())))
Wp32 = torch.zeros(32, C, device=dev, dtype=torch.bfloat16)
Wp32[:K] = Wb
print("bf16 mm padded K=32       %.1f us" % t(lambda: torch.mm(h, Wp32.t())))
gb = g.to(torch.bfloat16)
print("dW fp32 g^T h.float()     %.1f us" % t(lambda: g.t() @ h.float()))
print("dW bf16 g^T h             %.1f us" % t(lambda: gb.t() @ h))
