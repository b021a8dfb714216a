"""GPU: the fused pretraining heads + loss (HeadsLossFn: the one-launch local head of csrc/lhead.hip
for B <= 1024 (two positions per workgroup up to B = 512, one above) and its five-pass form,
the GO head fused into the MFMA GEMM of csrc/gemm.hip) match the PyTorch fp32 reference
(models/proteinbert.py heads_torch + train/losses.py) -- loss, dh, dg and every head parameter
gradient (Wo, bo, Wa, ba), at the real 8943-wide GO head and at batch / length extents that leave
partial 16-sample x 32-position tiles."""
import pytest
import torch

from proteinbert_pytorch_replication_amd.models import ProteinBERT
from proteinbert_pytorch_replication_amd.train.losses import pretrain_loss_torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,L,A", [(6, 24, 96), (100, 24, 96), (512, 24, 96), (640, 24, 96), (6, 1100, 96),
                                   (40, 2000, 96), (512, 64, 8943), (300, 37, 8943), (17, 512, 8943),
                                   (1024, 21, 96), (1030, 9, 96)])
@pytest.mark.parametrize("lhead_fused", [True, False])
def test_heads_loss_matches_torch(B, L, A, lhead_fused, monkeypatch):
    from proteinbert_pytorch_replication_amd.ops import global_track
    from proteinbert_pytorch_replication_amd.ops.global_track import HeadsLossFn
    monkeypatch.setattr(global_track, "LHEAD_FUSED", lhead_fused)
    torch.manual_seed(B + L)
    G = 256
    m = ProteinBERT(sequences_length=L, num_annotations=A, local_dim=128, global_dim=G, key_dim=64, num_heads=4,
                    num_blocks=1, device="cuda", backend="hip")
    h = torch.randn(B, L, 128, device="cuda").to(torch.bfloat16).requires_grad_(True)
    g = torch.randn(B, G, device="cuda").to(torch.bfloat16).float().requires_grad_(True)
    y_l = torch.randint(0, 26, (B, L), device="cuda")
    y_g = (torch.rand(B, A, device="cuda") < 0.05).float()
    w_l = (torch.rand(B, L, device="cuda") < 0.9).float()
    w_g = torch.ones(B, 1, device="cuda").expand(B, A)
    lo, go = m.pretraining_local_output[0], m.pretraining_global_output[0]
    total, parts = HeadsLossFn.apply(h, g, g.detach().to(torch.bfloat16), lo.weight, lo.bias, go.weight, go.bias,
                                     y_l, y_g, w_l, w_g)
    total.backward()
    got = {"h": h.grad.float().clone(), "g": g.grad.clone(), "wo": lo.weight.grad.clone(),
           "bo": lo.bias.grad.clone(), "wa": go.weight.grad.clone(), "ba": go.bias.grad.clone()}
    m.zero_grad(set_to_none=True)
    h2 = h.detach().float().requires_grad_(True)
    g2 = g.detach().clone().requires_grad_(True)
    pl, pg = m.heads_torch(h2, g2)
    ref_total = pretrain_loss_torch(pl, pg, {"local": y_l, "global": y_g}, {"local": w_l, "global": w_g})
    ref_total.backward()
    ref = {"h": h2.grad, "g": g2.grad, "wo": lo.weight.grad, "bo": lo.bias.grad, "wa": go.weight.grad,
           "ba": go.bias.grad}
    torch.cuda.synchronize()
    assert abs(total.item() - ref_total.item()) < 1e-3 * abs(ref_total.item())
    for k in ref:
        err = (got[k] - ref[k]).norm().item()
        print(f"B={B} L={L} A={A} {k:3s} |g| {ref[k].norm().item():.3e} err {err:.3e}")
        if k == "bo":
            # sum_b of a softmax over the batch axis: the exact gradient is 0; both sides
            # hold only summation noise, bounded by the scale of the weight gradient of the same head
            assert err < 1e-3 * ref["wo"].norm().item() + 1e-7
            continue
        assert err < 1e-2 * ref[k].norm().item() + 1e-7, f"B={B} {k}: err {err:.3e} |g| {ref[k].norm().item():.3e}"
