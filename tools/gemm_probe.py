"""Time candidate hipBLASLt formulations of the large-N / small-K head GEMMs (B=256, A=8943, G=512)."""
import torch, time
dev = "cuda"
B, A, G = 256, 8943, 512
bf = torch.bfloat16
dz = torch.randn(B, A, device=dev).to(bf)
g2 = torch.randn(B, G, device=dev).to(bf)
wa = torch.randn(A, G, device=dev).to(bf)
ann = (torch.rand(B, A, device=dev) < 0.01).to(bf)
du = torch.randn(B, G, device=dev).to(bf)
dwa = torch.zeros(A, G, device=dev)
dwin = torch.zeros(G, A, device=dev)

def t(fn, n=20):
    fn(); torch.cuda.synchronize()
    s = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - s) / n * 1e6

cands = {
 "dWA addmm(dwa, dz.t(), g2)": lambda: torch.addmm(dwa, dz.t(), g2, out_dtype=torch.float32, out=dwa),
 "dWA mm(dz.t(), g2)": lambda: torch.mm(dz.t(), g2, out_dtype=torch.float32),
 "dWA mm(dz.t().contig, g2)": lambda: torch.mm(dz.t().contiguous(), g2, out_dtype=torch.float32),
 "dWA^T mm(g2.t(), dz)": lambda: torch.mm(g2.t(), dz, out_dtype=torch.float32),
 "dWA^T mm(g2.t().contig, dz)": lambda: torch.mm(g2.t().contiguous(), dz, out_dtype=torch.float32),
 "dWA bf16 out mm(dz.t(), g2)": lambda: torch.mm(dz.t(), g2),
 "dWA^T addmm(dwin, g2.t(), dz)": lambda: torch.addmm(dwin, g2.t(), dz, out_dtype=torch.float32, out=dwin),
 "GO fwd mm(g2, wa.t())": lambda: torch.mm(g2, wa.t(), out_dtype=torch.float32),
 "dg2 mm(dz, wa)": lambda: torch.mm(dz, wa, out_dtype=torch.float32),
 "in fwd mm(ann, win.t())": lambda: torch.mm(ann, dwin.to(bf).t(), out_dtype=torch.float32),
 "dWin addmm(dwin, du.t(), ann)": lambda: torch.addmm(dwin, du.t(), ann, out_dtype=torch.float32, out=dwin),
 "dWin mm(du.t().contig, ann)": lambda: torch.mm(du.t().contiguous(), ann, out_dtype=torch.float32),
 "dWin^T mm(ann.t(), du)": lambda: torch.mm(ann.t(), du, out_dtype=torch.float32),
 "small 256x512x512": lambda: torch.mm(g2, wa[:512].t(), out_dtype=torch.float32),
 "small dW 512x512 K256": lambda: torch.mm(du.t(), g2, out_dtype=torch.float32),
}
for k, f in cands.items():
    try:
        print(f"{t(f):9.1f} us  {k}", flush=True)
    except Exception as e:
        print(f"   failed  {k}: {e}")
