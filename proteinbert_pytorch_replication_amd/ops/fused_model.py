"""HIP execution of the whole ProteinBERT forward (+ loss) on MI355X.

Reference forward: ``ProteinBERT/modules.py:295-304``; loss ``ProteinBERT/utils.py:293-294``.
The local track of every block runs as :class:`.local_track.LocalBlockFn` (fused CDNA4 kernels);
the embedding gather/scatter is a HIP kernel pair; the global track (``[B, 512]`` vectors, ~0.1 %
of FLOPs), the 8943-wide GO input/output GEMMs (hipBLASLt) and the heads run as PyTorch ops.
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
import torch.nn.functional as F

from .local_track import CH, EmbedFn, local_block
from ..train.losses import pretrain_loss_torch


def hip_supported(model) -> Tuple[bool, str]:
    cfg = model.config
    if cfg["local_dim"] != CH:
        return False, f"local_dim={cfg['local_dim']} (HIP kernels are specialised for 128)"
    if cfg["conv_kernel_size"] != 9:
        return False, f"conv_kernel_size={cfg['conv_kernel_size']} (HIP kernels are specialised for 9)"
    if cfg["vocab_size"] > 32:
        return False, "vocab_size > 32"
    if cfg["semantics"] != "reference":
        return False, "paper semantics run on the eager path"
    if (cfg["global_dim"] % 32) != 0:
        return False, "global_dim must be a multiple of 32"
    return True, ""


def _check(model) -> None:
    ok, why = hip_supported(model)
    if not ok:
        raise NotImplementedError(f"HIP backend: unsupported configuration: {why}")


def _gelu_linear(x: torch.Tensor, seq) -> torch.Tensor:
    lin = seq[0]
    return F.gelu(F.linear(x, lin.weight, lin.bias))


def fused_encode(model, tokens: torch.Tensor, annotations: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    _check(model)
    h = EmbedFn.apply(tokens, model.local_embedding.weight)                      # [B,L,128] bf16
    lin = model.global_linear_layer[0]
    g = F.gelu(F.linear(annotations.to(torch.bfloat16), lin.weight.to(torch.bfloat16),
                        lin.bias.to(torch.bfloat16))).float()                    # [B,G]
    for blk in model.proteinBERT_blocks:
        gb = _gelu_linear(g, blk.global_to_local_linear_layer)                   # [B,128]
        h, vpart = local_block(h, gb, blk)
        att = blk.global_attention_layer
        ga = vpart.sum(dim=1) * (att.W_parameter.sum() / att.key_dim)           # [B,G]
        n1, n2 = blk.global_norm_1, blk.global_norm_2
        g1 = F.layer_norm(g + _gelu_linear(g, blk.global_linear_layer_1) + ga, n1.normalized_shape, n1.weight,
                          n1.bias, n1.eps)
        g = F.layer_norm(g1 + _gelu_linear(g1, blk.global_linear_layer_2), n2.normalized_shape, n2.weight,
                         n2.bias, n2.eps)
    return h, g


def fused_forward(model, tokens: torch.Tensor, annotations: torch.Tensor):
    h, g = fused_encode(model, tokens, annotations)
    return model.heads_torch(h, g)


def fused_pretrain_loss(model, X: Dict[str, torch.Tensor], Y: Dict[str, torch.Tensor], W: Dict[str, torch.Tensor],
                        return_parts: bool = False):
    probs_l, probs_g = fused_forward(model, X["local"], X["global"])
    return pretrain_loss_torch(probs_l, probs_g, Y, {k: v.float() for k, v in W.items()}, model.semantics,
                               return_parts=return_parts)
