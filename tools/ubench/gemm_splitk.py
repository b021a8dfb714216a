"""Long-K GEMMs of the global input layer / GO head (K = 8943) on hipBLASLt: plain torch.mm vs split-K
as a batched GEMM + sum.   python tools/ubench/gemm_splitk.py"""
import torch

dev = torch.device("cuda")
bf = torch.bfloat16
B, G, A = 512, 512, 8943


def timeit(fn, n=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000.0


ann = (torch.rand(B, A, device=dev) < 0.005).to(bf)
w = (torch.randn(G, A, device=dev) * 0.01).to(bf)          # Linear weight [out, in]
ref = torch.mm(ann, w.t(), out_dtype=torch.float32)
print(f"input fwd  mm [B,A]x[A,G]: {timeit(lambda: torch.mm(ann, w.t(), out_dtype=torch.float32)):7.1f} us")
for S in (5, 9, 18, 35):
    Kc = (A + S - 1) // S
    Kp = Kc * S
    annp = torch.zeros(B, Kp, device=dev, dtype=bf); annp[:, :A] = ann
    wp = torch.zeros(G, Kp, device=dev, dtype=bf); wp[:, :A] = w
    a3 = annp.view(B, S, Kc).transpose(0, 1)                 # [S, B, Kc]
    b3 = wp.view(G, S, Kc).permute(1, 2, 0)                  # [S, Kc, G]
    f = lambda: torch.bmm(a3, b3, out_dtype=torch.float32).sum(0)
    err = (f() - ref).abs().max().item()
    print(f"input fwd  split-K S={S:2d} (strided views): {timeit(f):7.1f} us  maxerr {err:.2e}")
    a3c, b3c = a3.contiguous(), b3.contiguous()
    f2 = lambda: torch.bmm(a3c, b3c, out_dtype=torch.float32).sum(0)
    print(f"input fwd  split-K S={S:2d} (contiguous):    {timeit(f2):7.1f} us")
# GO head backward dX = dlogits [B, A] x W_go [A, G]
dl = (torch.randn(B, A, device=dev) * 1e-3).to(bf)
wgo = (torch.randn(A, G, device=dev) * 0.01).to(bf)
print(f"GO dX      mm [B,A]x[A,G]: {timeit(lambda: torch.mm(dl, wgo, out_dtype=torch.float32)):7.1f} us")
for S in (9, 18):
    Kc = (A + S - 1) // S
    Kp = Kc * S
    dlp = torch.zeros(B, Kp, device=dev, dtype=bf); dlp[:, :A] = dl
    wgp = torch.zeros(Kp, G, device=dev, dtype=bf); wgp[:A] = wgo
    a3 = dlp.view(B, S, Kc).transpose(0, 1)
    b3 = wgp.view(S, Kc, G)
    f = lambda: torch.bmm(a3, b3, out_dtype=torch.float32).sum(0)
    print(f"GO dX      split-K S={S:2d}: {timeit(f):7.1f} us")
# weight gradients (K = B = 512): dW_in = du^T ann, dW_go = dlogits^T g
du = torch.randn(B, G, device=dev).to(bf)
dw = torch.zeros(G, A, device=dev)
print(f"input dW   addmm [G,B]x[B,A] into fp32: {timeit(lambda: torch.addmm(dw, du.t(), ann, out_dtype=torch.float32, out=dw)):7.1f} us")
g = torch.randn(B, G, device=dev).to(bf)
dwg = torch.zeros(A, G, device=dev)
print(f"GO dW      addmm [A,B]x[B,G] into fp32: {timeit(lambda: torch.addmm(dwg, dl.t(), g, out_dtype=torch.float32, out=dwg)):7.1f} us")
print(f"GO fwd     mm [B,G]x[G,A]: {timeit(lambda: torch.mm(g, wgo.t(), out_dtype=torch.float32)):7.1f} us")
