"""HIP execution of the whole ProteinBERT forward (+ loss) on MI355X.

Reference forward: ``ProteinBERT/modules.py:295-304``; loss ``ProteinBERT/utils.py:293-294``.
Every piece runs on in-tree CDNA4 HIP kernels (``csrc/*.hip``), none on library GEMMs:
the local track of a block is :class:`.local_track.LocalBlockFn` (reference semantics) or
:class:`.paper_track.PaperBlockFn` (paper semantics); the global track is one fused forward and one
fused backward launch per block (:class:`.global_track.FusedGlobalBlockFn`, ``csrc/glob3.hip`` /
``csrc/glob2.hip``); the multi-hot GO input layer is a CSR embedding-bag (``csrc/annot.hip``); the
embedding is a gather/one-hot-GEMM pair; the heads + loss are ``csrc/lhead.hip`` (reference) /
``csrc/phead.hip`` (paper) and the fused GO head in ``csrc/gemm.hip``.
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
import torch.nn.functional as F

from .global_track import FusedGlobalBlockFn, GlobalBlockFn, HeadsLossFn, InputLayerFn, glob_fused_ok, pack_batch
from . import local_track as _lt
from .local_track import CH, EmbedFn, conv_images, embed_tokens, local_block, wgrad_tok_ok
from .paper_track import PaperHeadsLossFn, paper_block, unit_attention_weight


def hip_supported(model) -> Tuple[bool, str]:
    cfg = model.config
    if cfg["local_dim"] != CH:
        return False, f"local_dim={cfg['local_dim']} (HIP kernels are specialised for 128)"
    if cfg["conv_kernel_size"] != 9:
        return False, f"conv_kernel_size={cfg['conv_kernel_size']} (HIP kernels are specialised for 9)"
    if cfg["vocab_size"] > 32:
        return False, "vocab_size > 32"
    if cfg["semantics"] == "paper":
        from .paper_attention import KEY_DIM, VALUE_DIM
        if cfg["key_dim"] != KEY_DIM or cfg["global_dim"] // cfg["num_heads"] != VALUE_DIM:
            return False, (f"paper semantics: the HIP attention core is built for key_dim={KEY_DIM}, "
                           f"value_dim={VALUE_DIM}")
    if (cfg["global_dim"] % 32) != 0:
        return False, "global_dim must be a multiple of 32"
    return True, ""


def _check(model) -> None:
    ok, why = hip_supported(model)
    if not ok:
        raise NotImplementedError(f"HIP backend: unsupported configuration: {why}")


def fused_encode(model, tokens: torch.Tensor, annotations: torch.Tensor,
                 return_bf16: bool = False, cp=None):
    """Encoder on the HIP path: returns ``h [B, L, 128]`` (bf16) and ``g [B, G]`` (fp32).

    ``cp`` (:class:`..parallel.cp_fused.CPShard`): ``tokens`` is this rank's slice of the sequence;
    the local track runs on the slice (halo rows and LayerNorm statistics exchanged inside the block),
    the global track is replicated from the group-wide attention-pool sum."""
    _check(model)
    if cp is None:
        model.check_length(tokens.shape[1])   # the kernels index the [L, C] LayerNorm affine by position
    else:
        model.check_length(cp.L)
        if tokens.shape[1] != cp.shard_len:
            raise ValueError(f"expected a {cp.shard_len}-residue shard, got {tokens.shape[1]}")
    blocks = list(model.proteinBERT_blocks)
    lin = model.global_linear_layer[0]
    gl0 = blocks[0].global_to_local_linear_layer[0]
    # g0 and block 0's global->local vector; every GlobalBlockFn then produces the next block's gb
    g, g_bf, gb = InputLayerFn.apply(annotations, lin.weight, lin.bias, gl0.weight, gl0.bias)
    paper = model.semantics == "paper"
    emb_w = model.local_embedding.weight
    tok_c = tokens.contiguous()
    # the first block folds its conv data gradient into the embedding gradient (local_track.EMBED_FOLD)
    fold = (_lt.EMBED_FOLD and cp is None and tokens.device.type == "cuda" and len(blocks) > 0
            and wgrad_tok_ok(tok_c, emb_w, tokens.shape[1], blocks[0].local_narrow_conv_layer[0].weight.shape[2]))
    # [B,L,128] bf16; reference semantics folded: no embedding tensor at all, the first conv gathers
    # emb[tok] in its staging pass (pbx_conv_fwd3t)
    if fold and not paper and _lt.EMBED_GATHER:
        h = None
    else:
        h = embed_tokens(tok_c, emb_w) if fold else EmbedFn.apply(tokens, emb_w)
    mask = (tokens != 0).contiguous() if paper else None
    # every weight image the fused kernels read this step, built by one launch
    items, conv_imgs, glob_imgs = [], [], []
    for i, blk in enumerate(blocks):
        imgs, it = conv_images(blk.local_narrow_conv_layer[0].weight, blk.local_wide_conv_layer[0].weight)
        conv_imgs.append(imgs)
        items += it
        nxt = blocks[i + 1].global_to_local_linear_layer[0] if i + 1 < len(blocks) else None
        if glob_fused_ok(g.shape[1], 0 if nxt is None else nxt.weight.shape[0]):
            ws = [blk.global_linear_layer_1[0].weight, blk.global_linear_layer_2[0].weight,
                  None if nxt is None else nxt.weight]
            imgs = []
            for w in ws:
                if w is None:
                    imgs += [None, None]
                    continue
                o1, o2 = (torch.empty(w.numel(), dtype=torch.bfloat16, device=w.device) for _ in range(2))
                imgs += [o1, o2]
                items.append((1, w.detach(), o1, o2, w.shape[0], w.shape[1]))
            glob_imgs.append(tuple(imgs))
        else:
            glob_imgs.append(None)
    pack_batch(items)
    for i, blk in enumerate(blocks):
        att = blk.global_attention_layer
        if paper:
            # per-position LayerNorm local track, then attention over positions (split-L HIP core);
            # its [B, G] output enters the global track unscaled (W_parameter unused, as in the oracle)
            first = i == 0 and cp is None
            h, o = paper_block(h, gb, g, blk, mask, conv_imgs[i], tok=tok_c if first else None,
                               emb=emb_w if first else None, emb_grad=fold and i == 0, cp=cp)
            vpart = o.unsqueeze(1)
            wp = unit_attention_weight(att.key_dim, h.device)
        else:
            # the first block's input is the embedding: its conv weight gradient goes through the tokens
            first = i == 0 and cp is None
            h, vpart = local_block(h, gb, blk, conv_imgs[i], tail=(i == 0), cp=cp,
                                   tok=tok_c if first else None, emb=emb_w if first else None,
                                   emb_grad=fold and i == 0)
            if cp is not None:
                vpart = cp.pool_sum(vpart)      # [B, 1, NJ]: the group-wide sum over every shard's tiles
            wp = att.W_parameter
        nxt = blocks[i + 1].global_to_local_linear_layer[0] if i + 1 < len(blocks) else None
        l1, l2 = blk.global_linear_layer_1[0], blk.global_linear_layer_2[0]
        n1, n2 = blk.global_norm_1, blk.global_norm_2
        args = (g, g_bf, vpart, l1.weight, l1.bias, n1.weight, n1.bias, l2.weight, l2.bias, n2.weight, n2.bias,
                wp, None if nxt is None else nxt.weight, None if nxt is None else nxt.bias)
        if glob_imgs[i] is not None:
            g, g_bf, gb = FusedGlobalBlockFn.apply(*args, glob_imgs[i])
        else:
            g, g_bf, gb = GlobalBlockFn.apply(*args)
    if return_bf16:
        return h, g, g_bf
    return h, g


def fused_forward(model, tokens: torch.Tensor, annotations: torch.Tensor):
    h, g = fused_encode(model, tokens, annotations)
    return model.heads_torch(h, g)


def fused_pretrain_loss(model, X: Dict[str, torch.Tensor], Y: Dict[str, torch.Tensor], W: Dict[str, torch.Tensor],
                        return_parts: bool = False, cp=None):
    """Reference loss (utils.py:293-294) through the fused heads: one HIP pass per head.  With ``cp`` the
    local inputs / targets / weights are this rank's slice and the local (CE) term is this rank's share
    of the group's mean over B * L (see :mod:`..parallel.cp_fused`)."""
    h, g, g_bf = fused_encode(model, X["local"], X["global"], return_bf16=True, cp=cp)
    if cp is not None:
        W = dict(W, local=W["local"].float() * (cp.shard_len / cp.L))
    lo, go = model.pretraining_local_output[0], model.pretraining_global_output[0]
    fn = PaperHeadsLossFn if model.semantics == "paper" else HeadsLossFn
    total, parts = fn.apply(h, g, g_bf, lo.weight, lo.bias, go.weight, go.bias, Y["local"], Y["global"],
                                     W["local"], W["global"])
    if return_parts:
        return total, parts[0], parts[1]
    return total
