"""Microbenchmark of the in-tree MFMA GEMM (ops/gemm.py) per layout / shape / split vs torch.mm."""
import sys
import torch
sys.path.insert(0, ".")
from proteinbert_pytorch_replication_amd.ops.gemm import gemm  # noqa: E402


def t_us(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return 1000 * e0.elapsed_time(e1) / n


for (M, N, K) in [(512, 512, 512), (128, 512, 512), (512, 512, 4096), (512, 8943, 512)]:
    for ta, tb in [(False, True), (False, False), (True, False), (True, True)]:
        a = torch.randn((K, M) if ta else (M, K), device="cuda").to(torch.bfloat16)
        b = torch.randn((N, K) if tb else (K, N), device="cuda").to(torch.bfloat16)
        out = torch.empty(M, N, device="cuda")
        ao = a.t() if ta else a
        bo = b.t() if tb else b
        res = [f"M={M} N={N} K={K} ta={int(ta)} tb={int(tb)}"]
        for s in (1, 2, 4, 8):
            res.append(f"s{s} {t_us(lambda: gemm(a, b, out, ta, tb, splitk=s)):.1f}")
        res.append(f"torch.mm {t_us(lambda: torch.mm(ao, bo, out_dtype=torch.float32)):.1f}")
        print("  ".join(res), flush=True)
