"""Time the fp32 query-path GEMMs (csrc/sgemm.hip) at the paper config: B=1024, G=512, H=4, Kd=64."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from proteinbert_pytorch_replication_amd.ops import _lib, paper_track  # noqa: E402,F401

B, G, H, Kd = 1024, 512, 4, 64
dev = torch.device("cuda")
st = _lib.stream_ptr(dev)
g = torch.randn(B, G, device=dev)
wq = torch.randn(H, G, Kd, device=dev) * 0.05
q, qs, dqs = (torch.randn(B, H * Kd, device=dev) for _ in range(3))
dg = torch.empty(B, G, device=dev)
dwq = torch.zeros(H, G, Kd, device=dev)
s = 0.125
ws = torch.empty(_lib.lib().pbx_sg_query_ws(B, G, H, Kd), device=dev)
calls = {
    "fwd": lambda: _lib.call("pbx_sg_query_fwd", g.data_ptr(), wq.data_ptr(), q.data_ptr(), qs.data_ptr(), ws.data_ptr(), B, G, H, Kd, s, st),
    "dg": lambda: _lib.call("pbx_sg_query_dg", dqs.data_ptr(), q.data_ptr(), wq.data_ptr(), dg.data_ptr(), ws.data_ptr(), B, G, H, Kd, s, st),
    "dwq": lambda: _lib.call("pbx_sg_query_dwq", g.data_ptr(), dqs.data_ptr(), q.data_ptr(), dwq.data_ptr(), ws.data_ptr(), B, G, H, Kd, s, st),
}
for name, fn in calls.items():
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) / 20 * 1000:.1f} us", flush=True)
