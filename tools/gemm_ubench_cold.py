"""In-tree GEMM with cold operands (an L2/MALL flush between launches), accumulate into an fp32 output:
the conditions of the step's weight-gradient GEMMs."""
import sys
import torch
sys.path.insert(0, ".")
from proteinbert_pytorch_replication_amd.ops.gemm import gemm  # noqa: E402

flush = torch.empty(512 * 2**20, dtype=torch.uint8, device="cuda")


def t_us(fn, n=20):
    ts = []
    for i in range(n + 3):
        flush.add_(1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if i >= 3:
            ts.append(1000 * e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


for (M, N, K) in [(512, 512, 512), (128, 512, 512), (512, 8943, 512)]:
    for ta, tb in [(True, False), (False, False), (False, True)]:
        a = torch.randn((K, M) if ta else (M, K), device="cuda").to(torch.bfloat16)
        b = torch.randn((N, K) if tb else (K, N), device="cuda").to(torch.bfloat16)
        out = torch.zeros(M, N, device="cuda")
        res = [f"M={M} N={N} K={K} ta={int(ta)} tb={int(tb)}"]
        for s in (1, 2, 4):
            res.append(f"s{s} {t_us(lambda: gemm(a, b, out, ta, tb, splitk=s, accumulate=True)):.1f}")
        res.append(f"noacc-s1 {t_us(lambda: gemm(a, b, out, ta, tb, splitk=1)):.1f}")
        ao = a.t() if ta else a
        bo = b.t() if tb else b
        res.append(f"torch.mm {t_us(lambda: torch.mm(ao, bo, out_dtype=torch.float32)):.1f}")
        res.append(f"empty-event {t_us(lambda: None):.1f}")
        print("  ".join(res), flush=True)
