"""Loss precision vs the reference: the reference keeps the per-residue / per-annotation
loss weights in float64 (data_processing.py:175-176), so its loss reduction runs in float64
(utils.py:293-294); the fused HIP heads reduce in fp32.  These tests bound what that changes.

* CPU: the same probabilities and targets, weights in float32 vs float64, at the headline shape's element
  count per GPU step (B x L = 1024 x 512 residues, 8943 annotations x 1024): the two losses differ by < 1e-6
  relative -- far below the bf16 compute differences of the fused path.
* GPU: the fused HIP loss vs the fp32 PyTorch model with float64 weights (float64 loss reduction)."""
import pytest
import torch

from proteinbert_pytorch_replication_amd.train.losses import pretrain_loss_torch


def test_fp32_vs_float64_loss_reduction_cpu():
    g = torch.Generator().manual_seed(0)
    B, L, V, A = 1024, 512, 26, 8943
    logits = torch.randn(B, L, V, generator=g)
    probs_l = torch.softmax(logits, dim=0)             # reference semantics: softmax over the batch axis
    probs_g = torch.sigmoid(torch.randn(B, A, generator=g))
    Y = {"local": torch.randint(0, V, (B, L), generator=g), "global": (torch.rand(B, A, generator=g) < 0.01)}
    w_l = (torch.rand(B, L, generator=g) < 0.9).double()
    w_g = torch.ones(B, A, dtype=torch.float64)
    l64 = pretrain_loss_torch(probs_l, probs_g, Y, {"local": w_l, "global": w_g})
    l32 = pretrain_loss_torch(probs_l, probs_g, Y, {"local": w_l.float(), "global": w_g.float()})
    assert l64.dtype == torch.float64 and l32.dtype == torch.float32
    rel = abs(float(l32) - float(l64)) / abs(float(l64))
    print(f"fp32 vs float64 loss reduction: rel {rel:.2e}")
    assert rel < 1e-6


@pytest.mark.gpu
def test_fused_loss_vs_float64_reference_gpu():
    from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
    from proteinbert_pytorch_replication_amd.models import ProteinBERT
    from proteinbert_pytorch_replication_amd.ops.fused_model import fused_pretrain_loss
    torch.manual_seed(3)
    L, A, B = 512, 8943, 64
    m = ProteinBERT(sequences_length=L, num_annotations=A, local_dim=128, global_dim=512, key_dim=64, num_heads=4,
                    num_blocks=2, device="cuda", backend="hip")
    X, Y, W = SyntheticUniRefGO(L, A, B, "cuda", seed=9).next_batch()
    with torch.no_grad():
        fused = float(fused_pretrain_loss(m, X, Y, W))
        h, gl = m.encode_torch(X["local"], X["global"], torch.float32)
        pl, pg = m.heads_torch(h, gl)
        ref = pretrain_loss_torch(pl.double(), pg.double(), Y, {k: v.double() for k, v in W.items()})
    assert ref.dtype == torch.float64
    rel = abs(fused - float(ref)) / abs(float(ref))
    print(f"fused fp32-reduced loss {fused:.6f} vs float64 reference {float(ref):.6f}: rel {rel:.2e}")
    assert rel < 3e-3
