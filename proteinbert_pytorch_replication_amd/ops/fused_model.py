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

from .global_track import GlobalBlockFn, HeadsLossFn, InputLayerFn
from .local_track import CH, EmbedFn, local_block


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


def fused_encode(model, tokens: torch.Tensor, annotations: torch.Tensor,
                 return_bf16: bool = False):
    """Encoder on the HIP path: returns ``h [B, L, 128]`` (bf16) and ``g [B, G]`` (fp32)."""
    _check(model)
    blocks = list(model.proteinBERT_blocks)
    lin = model.global_linear_layer[0]
    gl0 = blocks[0].global_to_local_linear_layer[0]
    # g0 and block 0's global->local vector; every GlobalBlockFn then produces the next block's gb
    g, g_bf, gb = InputLayerFn.apply(annotations, lin.weight, lin.bias, gl0.weight, gl0.bias)
    h = EmbedFn.apply(tokens, model.local_embedding.weight)                      # [B,L,128] bf16
    for i, blk in enumerate(blocks):
        h, vpart = local_block(h, gb, blk)
        att = blk.global_attention_layer
        nxt = blocks[i + 1].global_to_local_linear_layer[0] if i + 1 < len(blocks) else None
        l1, l2 = blk.global_linear_layer_1[0], blk.global_linear_layer_2[0]
        n1, n2 = blk.global_norm_1, blk.global_norm_2
        g, g_bf, gb = GlobalBlockFn.apply(g, g_bf, vpart, l1.weight, l1.bias, n1.weight, n1.bias, l2.weight, l2.bias,
                                          n2.weight, n2.bias, att.W_parameter,
                                          None if nxt is None else nxt.weight, None if nxt is None else nxt.bias)
    if return_bf16:
        return h, g, g_bf
    return h, g


def fused_forward(model, tokens: torch.Tensor, annotations: torch.Tensor):
    h, g = fused_encode(model, tokens, annotations)
    return model.heads_torch(h, g)


def fused_pretrain_loss(model, X: Dict[str, torch.Tensor], Y: Dict[str, torch.Tensor], W: Dict[str, torch.Tensor],
                        return_parts: bool = False):
    """Reference loss (utils.py:293-294) through the fused heads: one HIP pass per head."""
    h, g, g_bf = fused_encode(model, X["local"], X["global"], return_bf16=True)
    lo, go = model.pretraining_local_output[0], model.pretraining_global_output[0]
    total, parts = HeadsLossFn.apply(h, g, g_bf, lo.weight, lo.bias, go.weight, go.bias, Y["local"], Y["global"],
                                     W["local"], W["global"])
    if return_parts:
        return total, parts[0], parts[1]
    return total
