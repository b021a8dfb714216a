import torch, time
R, C, N = 512*512, 128, 768
h = torch.randn(R, C, device="cuda").to(torch.bfloat16)
d = torch.randn(R, N, device="cuda").to(torch.bfloat16)
def t(f, n=20):
    f(); torch.cuda.synchronize(); t0=time.perf_counter()
    for _ in range(n): f()
    torch.cuda.synchronize(); return (time.perf_counter()-t0)/n*1e6
for nc in (16, 32, 64, 128, 256, 512):
    f = lambda: torch.bmm(h.view(nc, -1, C).transpose(1, 2), d.view(nc, -1, N), out_dtype=torch.float32).sum(0)
    print("nc", nc, "%.1f us" % t(f))
# transposed storage variant: (d^T h)^T
for nc in (32, 64, 128):
    f = lambda: torch.bmm(d.view(nc, -1, N).transpose(1, 2), h.view(nc, -1, C), out_dtype=torch.float32).sum(0)
    print("nc T", nc, "%.1f us" % t(f))
print("mm full", "%.1f us" % t(lambda: torch.mm(h.t(), d, out_dtype=torch.float32)))
wc = torch.randn(C, N, device="cuda").to(torch.bfloat16)
print("pre mm", "%.1f us" % t(lambda: torch.mm(h, wc)))
print("dh mm", "%.1f us" % t(lambda: torch.mm(d, wc.t())))
print("dh mm fp32out", "%.1f us" % t(lambda: torch.mm(d, wc.t(), out_dtype=torch.float32)))
