"""GELU-core probe for tests/test_gpu_gelu_modes.py: run in a fresh process (the kernel library is loaded once per
process) with PBX_GELU=fitted|exact; prints one JSON line.

* ``vpart``: the attention-pool forward (csrc/pool.hip) sums GELU(h2 Wv) over 32-position tiles in fp32 -- with
  h2 taken from the kernel's own bf16 output the only approximation left is the GELU core, so this isolates it;
* ``dh2``: the pool backward (GELU' recomputed), relative to its max;
* ``loss`` / ``grad``: a 2-block paper-config model, fused loss and gradients against the fp32 PyTorch oracle
  (exact nn.GELU): relative loss error and the worst per-parameter err / bound ratio (bf16 activations dominate).
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from proteinbert_pytorch_replication_amd.ops import _lib  # noqa: E402
from proteinbert_pytorch_replication_amd.ops import local_track  # noqa: E402,F401  (registers the launchers)


def pool_errors():
    dev = torch.device("cuda")
    st = _lib.stream_ptr(dev)
    B, L, NJ, C = 2, 512, 512, 128
    torch.manual_seed(7)
    TW = L // 32
    s2 = (torch.randn(B, L, C, device=dev) * 2 + 0.3).to(torch.bfloat16)
    st2 = torch.empty(B, TW, 2, device=dev)
    for t in range(TW):
        x = s2.float()[:, 32 * t:32 * t + 32].reshape(B, -1)
        st2[:, t, 0] = x.mean(1)
        st2[:, t, 1] = ((x - x.mean(1, keepdim=True)) ** 2).sum(1)
    g2 = torch.randn(L, C, device=dev) * 0.3 + 1
    be2 = torch.randn(L, C, device=dev) * 0.2
    wv = (torch.randn(NJ, C, device=dev) * 0.15).to(torch.bfloat16)
    h2 = torch.empty_like(s2)
    vpart = torch.empty(B, TW, NJ, device=dev)
    _lib.call("pbx_pool_fwd", s2.data_ptr(), st2.data_ptr(), g2.data_ptr(), be2.data_ptr(), wv.data_ptr(),
              h2.data_ptr(), vpart.data_ptr(), B, L, NJ, 1e-5, st)
    z = h2.double() @ wv.double().t()
    vr = F.gelu(z).view(B, TW, 32, NJ).sum(2)
    dv = torch.randn(B, NJ, device=dev) * 0.1
    dh2 = torch.empty_like(s2)
    sums2 = torch.empty(B, TW, 2, device=dev)
    _lib.call("pbx_pool_bwd", h2.data_ptr(), g2.data_ptr(), be2.data_ptr(), None, dv.data_ptr(), 1, wv.data_ptr(),
              dh2.data_ptr(), sums2.data_ptr(), B, L, NJ, st)
    torch.cuda.synchronize()
    gd = 0.5 * (1 + torch.erf(z / 2 ** 0.5)) + z * torch.exp(-0.5 * z * z) / (2 * torch.pi) ** 0.5
    dr = (gd * dv.double()[:, None, :]) @ wv.double()
    return (((vpart.double() - vr).abs().max() / vr.abs().max()).item(),
            ((dh2.double() - dr).abs().max() / dr.abs().max()).item())


def model_errors():
    from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
    from proteinbert_pytorch_replication_amd.models import ProteinBERT
    from proteinbert_pytorch_replication_amd.ops.fused_model import fused_pretrain_loss
    from proteinbert_pytorch_replication_amd.train.losses import pretrain_loss_torch
    torch.manual_seed(0)
    L, A = 256, 8943
    m = ProteinBERT(sequences_length=L, num_annotations=A, local_dim=128, global_dim=512, key_dim=64, num_heads=4,
                    num_blocks=2, device="cuda", backend="hip")
    X, Y, W = SyntheticUniRefGO(L, A, 6, "cuda", seed=3).next_batch()
    loss = fused_pretrain_loss(m, X, Y, W)
    loss.backward()
    got = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    m.zero_grad(set_to_none=True)
    h, g = m.encode_torch(X["local"], X["global"], torch.float32)
    pl, pg = m.heads_torch(h, g)
    lref = pretrain_loss_torch(pl, pg, Y, {k: v.float() for k, v in W.items()})
    lref.backward()
    torch.cuda.synchronize()
    # the bound of tests/test_hip_local_track.py: err < 3e-2 |g| + 1e-4 median|g| (the local-output bias has an
    # exact gradient of 0); reported as the worst ratio err / bound
    norms = {n: p.grad.norm().item() for n, p in m.named_parameters() if p.grad is not None}
    scale = sorted(norms.values())[len(norms) // 2]
    worst = 0.0
    for n, p in m.named_parameters():
        if p.grad is None:
            continue
        err = (got[n].float() - p.grad.float()).norm().item()
        worst = max(worst, err / (3e-2 * norms[n] + 1e-4 * scale))
    return abs(loss.item() - lref.item()) / abs(lref.item()), worst


if __name__ == "__main__":
    ev, ed = pool_errors()
    el, eg = model_errors()
    print(json.dumps({"mode": _lib.gelu_mode(), "lib": os.path.basename(_lib.HIP_LIB), "vpart": ev, "dh2": ed,
                      "loss": el, "grad": eg}), flush=True)
