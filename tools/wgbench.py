"""Weight-gradient kernel alone (csrc/wgrad.hip) at the paper config, for PMC passes:
    rocprofv3 --pmc ... -- python3 tools/wgbench.py [--B 512] [--R 64] [--iters 5]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from proteinbert_pytorch_replication_amd.ops import _lib  # noqa: E402
from proteinbert_pytorch_replication_amd.ops import local_track  # noqa: E402,F401  (registers the symbols)

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=512)
ap.add_argument("--L", type=int, default=512)
ap.add_argument("--R", type=int, default=64)
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
B, L, C, KS, dil, R = a.B, a.L, 128, 9, 5, a.R
dev = torch.device("cuda")
st = _lib.stream_ptr(dev)
bf = torch.bfloat16
x, dn, dw = ((torch.randn(B, L, C, device=dev) * 0.5).to(bf) for _ in range(3))
w0, w1 = torch.zeros(C, C, KS, device=dev), torch.zeros(C, C, KS, device=dev)
b0, b1 = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
slab = torch.empty(R, 2, KS, C, C, device=dev)
bslab = torch.empty(R, 2, C, device=dev)
for _ in range(a.iters):
    _lib.call("pbx_wgrad2", dn.data_ptr(), dw.data_ptr(), x.data_ptr(), slab.data_ptr(), bslab.data_ptr(),
              w0.data_ptr(), w1.data_ptr(), b0.data_ptr(), b1.data_ptr(), B, L, dil, 2, R, st)
torch.cuda.synchronize()
print("ok", float(w0.abs().sum()))
