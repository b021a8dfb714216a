"""The step's in-tree GEMMs at their real shapes / layouts / padding, cold operands (a 512 MB flush
between launches), accumulate as in the step; median event time.  Prints per-split timings."""
import sys
import torch
sys.path.insert(0, ".")
from proteinbert_pytorch_replication_amd.ops.gemm import gemm, split_count  # noqa: E402

dev = torch.device("cuda")
flush = torch.empty(512 * 2**20, dtype=torch.uint8, device=dev)
B, G, A, AP = 512, 512, 8943, 8960


def t_us(fn, n=15):
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


def bf(*s):
    return torch.randn(*s, device=dev).to(torch.bfloat16)


def padded(rows, cols, ld):
    buf = torch.zeros(rows, ld, device=dev, dtype=torch.bfloat16)
    buf[:, :cols] = bf(rows, cols)
    return buf[:, :cols]


ann = padded(B, A, AP)
dz = padded(B, A, AP)
du = bf(B, G)
g2 = bf(B, G)
wa = bf(A, G)
w_in = bf(G, A)
cases = {
    "dW_in += du^T ann   (M=512 N=8943 K=512, ta tb=0)": (du, ann, torch.zeros(G, A, device=dev), True, False, True, dict(pad_b=True)),
    "dWa += dz^T g2      (M=8943 N=512 K=512, ta tb=0)": (dz, g2, torch.zeros(A, G, device=dev), True, False, True, dict(pad_a=True)),
    "dg2 = dz Wa         (M=512 N=512 K=8943, ta=0 tb=0)": (dz, wa, torch.zeros(B, G, device=dev), False, False, False, dict(pad_a=True)),
    "u = ann W_in^T      (M=512 N=512 K=8943, ta=0 tb=1)": (ann, w_in, torch.zeros(B, G, device=dev), False, True, False, dict(pad_a=True)),
    "dW = du^T g         (M=512 N=512 K=512, ta tb=0)": (du, g2, torch.zeros(G, G, device=dev), True, False, True, {}),
}
for name, (a, b, out, ta, tb, acc, kw) in cases.items():
    M = a.shape[1] if ta else a.shape[0]
    K = a.shape[0] if ta else a.shape[1]
    N = b.shape[0] if tb else b.shape[1]
    res = [f"{name}: auto split {split_count(M, N, K, dev)}"]
    for s in (1, 2, 4, 8):
        res.append(f"s{s} {t_us(lambda: gemm(a, b, out, ta, tb, accumulate=acc, splitk=s, **kw)):.1f}")
    res.append(f"auto {t_us(lambda: gemm(a, b, out, ta, tb, accumulate=acc, **kw)):.1f}")
    ao = a.t() if ta else a
    bo = b.t() if tb else b
    res.append(f"torch.mm {t_us(lambda: torch.mm(ao, bo, out_dtype=torch.float32)):.1f}")
    print("  ".join(res), flush=True)
