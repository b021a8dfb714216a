"""Context (sequence) parallelism: shard the residue axis L of one batch across ranks.

The reference has no parallelism at all and one MI355X holds L=4096 comfortably
(§5.7), so this is the optional CP design of §2.4, built for runs whose per-sequence activations
outgrow one GPU or that want more GPUs on fewer sequences. Every rank holds the full (tiny, 16.8M)
parameter set and a contiguous slice ``[r*L/P, (r+1)*L/P)`` of every sequence; what couples the
slices inside a block (reference ``modules.py:201-231``) is:

* the narrow/wide dilated convs (``modules.py:124-147``): a halo of ``d*(k-1)/2`` residues (20 for
  k=9, d=5) from each neighbour — point-to-point send/recv, which on xGMI uses exactly one direct
  link per neighbour pair (no ring, no all-gather);
* ``LayerNorm((L, C))`` (``modules.py:148-151,212,217``, reference semantics): a per-sample
  two-pass (sum, then centred sum of squares) all-reduce of 2*B floats;
* the local->global attention (``modules.py:49-60``): reference semantics pools
  ``sum_l GELU(h Wv)`` -> one ``[B, G]`` all-reduce; paper semantics is split-L single-query
  attention -> all-reduce MAX of the row max, then SUM of ``(sum e^s v, sum e^s)`` partials.

The global track (``[B, G]``) is replicated: each rank recomputes it from identical inputs, which is
cheaper than broadcasting it. Every collective is differentiable (backward of a SUM all-reduce is a
SUM all-reduce of the incoming gradients, the halo exchange sends halo gradients back to their
owners), so ``sum_r loss_r`` is the single-device loss and summing parameter gradients over the
CP group gives its exact gradient: :func:`cp_pretrain_loss` weights the replicated GO term by
1/P for that reason, and :func:`all_reduce_grads` does the sum.

CP here runs the PyTorch op path (any dtype / device, paper semantics included); reference semantics on
the fused HIP executor is :mod:`.cp_fused` (the same collectives around the CDNA4 kernels).
Combine with data parallelism through :func:`make_cp_groups` (ranks ``[i*P, (i+1)*P)`` share
one batch; strided ranks form the DP groups).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.distributed.nn.functional as dfn
import torch.nn.functional as F

from ..models.proteinbert import ProteinBERT, ProteinBERTBlock, _gelu


def _group_rank_world(group) -> Tuple[int, int]:
    return dist.get_rank(group), dist.get_world_size(group)


def _peer(group, r: int) -> int:
    return dist.get_global_rank(group, r) if group is not None else r


def _exchange(send_left: Optional[torch.Tensor], send_right: Optional[torch.Tensor],
              recv_shape, dtype, device, group) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """Send ``send_left`` to rank-1 / ``send_right`` to rank+1; receive the matching strips."""
    rank, world = _group_rank_world(group)
    # gloo point-to-point does not order against the device stream: device strips go through host memory
    staged = torch.device(device).type == "cuda" and dist.get_backend(group) == "gloo"
    buf_dev = "cpu" if staged else device
    ops, from_left, from_right = [], None, None
    if rank > 0:
        from_left = torch.empty(recv_shape, dtype=dtype, device=buf_dev)
        ops.append(dist.P2POp(dist.isend, send_left.contiguous().to(buf_dev), _peer(group, rank - 1), group))
        ops.append(dist.P2POp(dist.irecv, from_left, _peer(group, rank - 1), group))
    if rank < world - 1:
        from_right = torch.empty(recv_shape, dtype=dtype, device=buf_dev)
        ops.append(dist.P2POp(dist.isend, send_right.contiguous().to(buf_dev), _peer(group, rank + 1), group))
        ops.append(dist.P2POp(dist.irecv, from_right, _peer(group, rank + 1), group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    if staged:
        from_left = None if from_left is None else from_left.to(device)
        from_right = None if from_right is None else from_right.to(device)
    return from_left, from_right


class _HaloExchange(torch.autograd.Function):
    """``[B, Ll, C]`` -> ``[B, Ll + 2*halo, C]`` with neighbours' edge residues (zeros at the
    sequence ends = the conv's ``padding="same"``). Backward returns halo gradients to their owners."""

    @staticmethod
    def forward(ctx, x, halo: int, group):
        ctx.halo, ctx.group = halo, group
        B, _, C = x.shape
        fl, fr = _exchange(x[:, :halo], x[:, -halo:], (B, halo, C), x.dtype, x.device, group)
        zeros = x.new_zeros(B, halo, C)
        return torch.cat([fl if fl is not None else zeros, x, fr if fr is not None else zeros], dim=1)

    @staticmethod
    def backward(ctx, gy):
        halo, group = ctx.halo, ctx.group
        B, _, C = gy.shape
        gx = gy[:, halo:-halo].contiguous().clone()
        # our left halo came from rank-1's right edge, our right halo from rank+1's left edge
        gl, gr = _exchange(gy[:, :halo], gy[:, -halo:], (B, halo, C), gy.dtype, gy.device, group)
        if gl is not None:
            gx[:, :halo] += gl
        if gr is not None:
            gx[:, -halo:] += gr
        return gx, None, None


def halo_exchange(x: torch.Tensor, halo: int, group=None) -> torch.Tensor:
    if x.shape[1] < halo:
        raise ValueError(f"context-parallel shard of {x.shape[1]} residues is shorter than the conv halo "
                         f"({halo}); use fewer CP ranks or a longer sequence")
    return _HaloExchange.apply(x, halo, group)


def _sum_all(t: torch.Tensor, group) -> torch.Tensor:
    return dfn.all_reduce(t, op=dist.ReduceOp.SUM, group=group)


class ContextParallelProteinBERT(torch.nn.Module):
    """Wraps a (replicated) :class:`ProteinBERT`; ``forward`` takes this rank's residue slice."""

    def __init__(self, model: ProteinBERT, group=None, compute_dtype: Optional[torch.dtype] = None):
        super().__init__()
        self.model = model
        self.group = group
        self.compute_dtype = compute_dtype
        self.rank, self.world = _group_rank_world(group)
        L = model.sequences_length
        if L % self.world:
            raise ValueError(f"sequences_length {L} is not divisible by the CP degree {self.world}")
        self.shard_len = L // self.world
        self.start = self.rank * self.shard_len
        blk: ProteinBERTBlock = model.proteinBERT_blocks[0]
        k, d = blk.conv_kernel_size, blk.wide_conv_dilation
        if k % 2 == 0:
            raise ValueError("context parallelism needs an odd conv kernel (symmetric 'same' padding)")
        self.pad_n, self.pad_w = (k - 1) // 2, d * (k - 1) // 2
        self.halo = max(self.pad_n, self.pad_w)

    # ---------------------------------------------------------------------------------------------
    def shard(self, t: torch.Tensor, dim: int = 1) -> torch.Tensor:
        """This rank's slice of a full-length ``[B, L, ...]`` tensor."""
        return t.narrow(dim, self.start, self.shard_len)

    def _conv(self, seq, ext: torch.Tensor, pad: int) -> torch.Tensor:
        conv = seq[0]
        lo = self.halo - pad
        x = ext[:, lo:lo + self.shard_len + 2 * pad].transpose(1, 2)
        y = F.conv1d(x, conv.weight.to(ext.dtype), conv.bias.to(ext.dtype), padding=0, dilation=conv.dilation)
        return _gelu(y.transpose(1, 2))

    def _local_norm(self, ln, x: torch.Tensor) -> torch.Tensor:
        if len(ln.normalized_shape) == 1:                       # paper semantics: per-residue LN over C
            return F.layer_norm(x.float(), ln.normalized_shape, ln.weight, ln.bias, ln.eps).to(x.dtype)
        xf = x.float()
        n = float(self.model.sequences_length * x.shape[2])
        mean = _sum_all(xf.sum(dim=(1, 2)), self.group) / n
        xc = xf - mean[:, None, None]
        var = _sum_all((xc * xc).sum(dim=(1, 2)), self.group) / n
        w = self.shard(ln.weight, 0)
        b = self.shard(ln.bias, 0)
        return (xc * torch.rsqrt(var + ln.eps)[:, None, None] * w + b).to(x.dtype)

    def _attention(self, att, h: torch.Tensor, g: torch.Tensor, mask: Optional[torch.Tensor]) -> torch.Tensor:
        if att.semantics != "paper":
            v = _gelu(torch.matmul(h, att.value_weight_cat().to(h.dtype)))
            return _sum_all(v.float().sum(dim=1), self.group) * (att.W_parameter.sum() / att.key_dim)
        q = torch.tanh(torch.einsum("bg,hgk->bhk", g, att.Wq.to(g.dtype)))
        k = torch.tanh(torch.einsum("blc,hck->bhlk", h, att.Wk.to(h.dtype)))
        v = _gelu(torch.einsum("blc,hcv->bhlv", h, att.Wv.to(h.dtype)))
        s = torch.einsum("bhk,bhlk->bhl", q.to(k.dtype), k).float() / (att.key_dim ** 0.5)
        if mask is not None:
            s = s.masked_fill(~mask.unsqueeze(1), float("-inf"))
        m = s.detach().amax(dim=-1)                              # softmax shift: no gradient needed
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=self.group)
        e = torch.exp(s - m.unsqueeze(-1))
        num = _sum_all(torch.einsum("bhl,bhlv->bhv", e, v.float()), self.group)
        den = _sum_all(e.sum(dim=-1), self.group)
        o = num / den.unsqueeze(-1)
        return o.reshape(o.shape[0], -1)

    def _block(self, blk: ProteinBERTBlock, h, g, mask):
        lin = lambda seq, x: _gelu(F.linear(x, seq[0].weight.to(x.dtype), seq[0].bias.to(x.dtype)))  # noqa: E731
        ext = halo_exchange(h, self.halo, self.group)
        n = self._conv(blk.local_narrow_conv_layer, ext, self.pad_n)
        w = self._conv(blk.local_wide_conv_layer, ext, self.pad_w)
        gb = lin(blk.global_to_local_linear_layer, g.to(h.dtype))
        h1 = self._local_norm(blk.local_norm_1, h + n + w + gb.unsqueeze(1))
        h2 = self._local_norm(blk.local_norm_2, h1 + lin(blk.local_linear_layer, h1))
        ga = self._attention(blk.global_attention_layer, h2, g, mask)
        gf = g.float()
        g1 = F.layer_norm(gf + lin(blk.global_linear_layer_1, gf) + ga, blk.global_norm_1.normalized_shape,
                          blk.global_norm_1.weight, blk.global_norm_1.bias, blk.global_norm_1.eps)
        g2 = F.layer_norm(g1 + lin(blk.global_linear_layer_2, g1), blk.global_norm_2.normalized_shape,
                          blk.global_norm_2.weight, blk.global_norm_2.bias, blk.global_norm_2.eps)
        return h2, g2

    def forward(self, tokens_local: torch.Tensor, annotations: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """``tokens_local`` ``[B, L/P]`` (this rank's slice), ``annotations`` ``[B, A]`` (full, replicated).

        Returns ``(probs_local [B, L/P, V], probs_global [B, A])`` — the slice of the single-device
        output and the (replicated) GO probabilities."""
        m = self.model
        if tokens_local.shape[1] != self.shard_len:
            raise ValueError(f"expected a {self.shard_len}-residue shard, got {tokens_local.shape[1]}")
        dt = self.compute_dtype or torch.float32
        h = m.local_embedding.weight.to(dt)[tokens_local]
        lin = m.global_linear_layer[0]
        g = _gelu(F.linear(annotations.to(dt), lin.weight.to(dt), lin.bias.to(dt))).float()
        mask = tokens_local != 0 if m.semantics == "paper" else None
        for blk in m.proteinBERT_blocks:
            h, g = self._block(blk, h, g, mask)
        return m.heads_torch(h, g)


def cp_pretrain_loss(probs_l: torch.Tensor, probs_g: torch.Tensor, y_local: torch.Tensor,
                     w_local: torch.Tensor, y_global: torch.Tensor, w_global: torch.Tensor,
                     seq_len: int, world: int, semantics: str = "reference") -> torch.Tensor:
    """This rank's share of the reference loss (``utils.py:293-294``): the CE sum over its residues
    divided by the full ``B*L``, plus 1/P of the replicated GO BCE mean. Summing over the CP group
    gives the single-device loss."""
    if semantics == "reference":
        ce = F.cross_entropy(probs_l.permute(0, 2, 1).float(), y_local, reduction="none")
    else:
        ce = F.nll_loss(torch.log(probs_l.float().clamp_min(1e-30)).permute(0, 2, 1), y_local, reduction="none")
    local = (ce * w_local).sum() / float(probs_l.shape[0] * seq_len)
    bce = F.binary_cross_entropy(probs_g.float(), y_global.float(), reduction="none")
    return local + torch.mean(bce * w_global) / world


def all_reduce_grads(params, group=None, average_over: Optional[int] = None) -> None:
    """Coalesced SUM all-reduce of parameter gradients over ``group`` (one flat buffer, one call);
    ``average_over`` divides afterwards (the DP factor when CP and DP share one group)."""
    grads: List[torch.Tensor] = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, group=group)
    if average_over:
        flat /= average_over
    o = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[o:o + n].view_as(g))
        o += n


def make_cp_groups(cp_size: int) -> Tuple[object, object]:
    """Split the world into CP groups of ``cp_size`` consecutive ranks (one xGMI hop between
    neighbours on a node) and DP groups of the strided ranks; returns ``(cp_group, dp_group)``
    for the calling rank. Every rank must call this (``new_group`` is collective)."""
    world, rank = dist.get_world_size(), dist.get_rank()
    if world % cp_size:
        raise ValueError(f"world size {world} is not divisible by cp_size {cp_size}")
    cp_group = dp_group = None
    for i in range(world // cp_size):
        g = dist.new_group(list(range(i * cp_size, (i + 1) * cp_size)))
        if rank // cp_size == i:
            cp_group = g
    for j in range(cp_size):
        g = dist.new_group(list(range(j, world, cp_size)))
        if rank % cp_size == j:
            dp_group = g
    return cp_group, dp_group


__all__ = ["ContextParallelProteinBERT", "halo_exchange", "cp_pretrain_loss", "all_reduce_grads", "make_cp_groups"]
