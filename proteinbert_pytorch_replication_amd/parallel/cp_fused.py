"""Context parallelism on the fused HIP executor (SURVEY §2.4 CP row, §5.7).

The residue axis L of every sequence is split over the ranks of a CP group; each rank runs the fused
CDNA4 local-track kernels on its slice ``[r L/P, (r+1) L/P)`` and the tiny global track replicated.
What couples the slices (reference ``ProteinBERT/modules.py:124-151,201-231``) and where it is
exchanged:

* the narrow / wide dilated convolutions need ``4 d`` = 20 neighbour rows on each side: the halo comes
  from the two ring neighbours by ``isend`` / ``irecv`` once per block and direction (``halo_rows`` /
  ``halo_rows_many``) and the conv kernels read it in place (``pbx_conv_fwd3x`` /
  ``pbx_wgrad2x`` take ``xlo`` / ``xhi`` halo rows; the data gradient ``pbx_conv_dgrad4x`` reads the
  neighbours' ``ds1`` and GELU' rows the same way, so no gradient is sent back);
* ``LayerNorm((L, C))`` statistics are per sample over the WHOLE sequence: the kernels' per-tile
  (mean, M2) partials are combined group-wide (one float64 all-reduce of (sum, sum of squares) per
  sample) and written back into the local partial table so that the unmodified kernels' Chan merge
  yields the global mean and variance (every tile gets the global mean and M2 / (P T)); the backward's
  (sum dxhat, sum dxhat xhat) partials are all-reduced the same way (local total = global / P, since the
  kernels divide by the local element count);
* the attention pool (reference semantics: a sum over positions) is all-reduced before the replicated
  global track, and the broadcast vector's gradient (a sum over positions) after the LayerNorm-1
  backward.

Gradient bookkeeping: every rank computes the EXACT gradient of the full loss with respect to the
replicated activations (the GO-head BCE is evaluated in full on every rank, the pool-sum and ``dgb``
collectives make the global track's inputs and upstream gradients group-wide) and with respect to its
own slice's activations (its share of the per-residue CE, normalised by the full ``B L``).  So the
local-track parameters (convs, [L, C] affine rows, local MLP, embedding, local head) hold per-shard
partial gradients that :func:`cp_reduce_grads` SUMs over the group, while the replicated parameters
(global track, GO input / output layers) already hold the full gradient on every rank.

Paper semantics (per-position LayerNorm, attention softmax over positions; ``ops/paper_track.py``) shards
the same way with less to exchange: no LayerNorm statistics, the conv halos as above, and the attention
over positions as a split softmax -- every rank's fused attention kernel covers its positions and the
group merges ``(o, logsumexp)`` (one MAX + one SUM all-reduce), after which the backward kernel is exact on
each shard; the query gradient and the broadcast vector's gradient are all-reduced.

Collectives are plain ``torch.distributed`` calls on the CP group (RCCL over xGMI on a node; gloo for
CPU rehearsal of the bookkeeping).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist


class CPShard:
    """This rank's place in a CP group and the collectives the fused local track calls."""

    def __init__(self, L: int, group=None, halo: int = 20):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if L % self.world:
            raise ValueError(f"sequence length {L} is not divisible by the CP degree {self.world}")
        self.L = L
        self.shard_len = L // self.world
        self.start = self.rank * self.shard_len
        self.halo = halo
        if self.shard_len < halo:
            raise ValueError(f"shard of {self.shard_len} residues is shorter than the conv halo ({halo})")

    # ---- helpers -------------------------------------------------------------------------------
    def shard(self, t: torch.Tensor, dim: int = 1) -> torch.Tensor:
        """This rank's slice of a full-length ``[B, L, ...]`` tensor (contiguous copy)."""
        return t.narrow(dim, self.start, self.shard_len).contiguous()

    def rows(self, t: torch.Tensor) -> torch.Tensor:
        """This rank's rows of an ``[L, C]`` LayerNorm affine (or its gradient): a contiguous view."""
        return t[self.start:self.start + self.shard_len]

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        dist.all_reduce(t, group=self.group)
        return t

    # ---- halo ----------------------------------------------------------------------------------
    def _peer(self, r: int) -> int:
        return r if self.group is None else dist.get_global_rank(self.group, r)

    def halo_rows_many(self, *xs: torch.Tensor) -> List[torch.Tensor]:
        """Each ``[B, Ls, C]`` -> ``[B, H + Ls + H, C]`` with the neighbours' edge rows (zeros beyond the
        sequence ends = the convs' ``padding="same"``).  Neighbour point-to-point only: one
        ``isend`` / ``irecv`` pair per neighbour carries the edge strips of every tensor (2 x B x H x C
        per tensor and direction, the same on every rank whatever the CP degree; on a node these are
        single-link xGMI transfers between ring neighbours)."""
        H = self.halo
        B, Ls, C = xs[0].shape
        for x in xs:
            if x.shape != (B, Ls, C) or x.dtype != xs[0].dtype:
                raise ValueError("halo_rows_many: tensors must share shape and dtype")
        n = len(xs)
        dev = xs[0].device
        lo = torch.stack([x[:, :H] for x in xs]).contiguous()            # [n, B, H, C] -> left neighbour
        hi = torch.stack([x[:, Ls - H:] for x in xs]).contiguous()       # -> right neighbour
        # gloo's point-to-point ops take the raw pointer and do not order against the device stream: a device
        # tensor could be read before the kernel producing it (or written before its zero-fill) ran, so gloo
        # groups (the one-GPU tests) stage the strips through host memory; RCCL orders them on its stream
        staged = dev.type == "cuda" and dist.get_backend(self.group) == "gloo"
        if staged:
            lo, hi = lo.cpu(), hi.cpu()
        left = torch.zeros_like(lo)
        right = torch.zeros_like(hi)
        ops = []
        if self.rank > 0:
            peer = self._peer(self.rank - 1)
            ops += [dist.P2POp(dist.isend, lo, peer, self.group), dist.P2POp(dist.irecv, left, peer, self.group)]
        if self.rank < self.world - 1:
            peer = self._peer(self.rank + 1)
            ops += [dist.P2POp(dist.isend, hi, peer, self.group), dist.P2POp(dist.irecv, right, peer, self.group)]
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        if staged:
            left, right = left.to(dev), right.to(dev)
        return [torch.cat([left[i], xs[i], right[i]], dim=1).contiguous() for i in range(n)]

    def halo_rows(self, x: torch.Tensor) -> torch.Tensor:
        """One tensor's halo exchange (:meth:`halo_rows_many`)."""
        return self.halo_rows_many(x)[0]

    # ---- LayerNorm((L, C)) statistics ----------------------------------------------------------
    def fix_stats(self, st: torch.Tensor, BM: int, C: int = 128) -> None:
        """``st [B, T, 2]``: per-tile (mean, M2) of this shard (tile t covers min(BM, Ls - t BM) rows).
        Rewritten in place so the kernels' combine gives the group-wide mean / variance."""
        B, T, _ = st.shape
        n_t = torch.tensor([min(BM, self.shard_len - t * BM) * C for t in range(T)], dtype=torch.float64,
                           device=st.device)
        m = st[..., 0].double()
        M2 = st[..., 1].double()
        n = float(self.shard_len * C)
        mean = (m * n_t).sum(dim=1) / n
        M2l = M2.sum(dim=1) + (n_t * (m - mean[:, None]) ** 2).sum(dim=1)
        s = torch.stack([n * mean, M2l + n * mean * mean], dim=1)                 # (sum, sum of squares)
        dist.all_reduce(s, group=self.group)
        ng = n * self.world
        mg = s[:, 0] / ng
        M2g = (s[:, 1] - ng * mg * mg).clamp_min(0.0)
        st[..., 0] = mg[:, None].to(st.dtype)
        st[..., 1] = (M2g / (self.world * T))[:, None].to(st.dtype)

    def fix_sums(self, sums: torch.Tensor) -> None:
        """``sums [B, T, 2]``: LayerNorm-backward partials (sum dxhat, sum dxhat xhat).  The kernels
        divide their total by the LOCAL element count, so the local total becomes group total / P."""
        tot = sums.double().sum(dim=1)
        dist.all_reduce(tot, group=self.group)
        tot /= self.world
        sums.zero_()
        sums[:, 0] = tot.to(sums.dtype)

    # ---- attention pool ------------------------------------------------------------------------
    def pool_sum(self, vpart: torch.Tensor) -> torch.Tensor:
        """``[B, T, NJ]`` per-tile pool partials -> ``[B, 1, NJ]`` group-wide sum (differentiable: the
        replicated global track hands every rank the gradient of the full loss, so the local pool's
        gradient is that same tensor -- the backward is the identity)."""
        return _PoolSum.apply(vpart, self)


class _PoolSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, vpart, cp: CPShard):
        out = vpart.sum(dim=1, keepdim=True).contiguous()
        dist.all_reduce(out, group=cp.group)
        ctx.T = vpart.shape[1]
        return out

    @staticmethod
    def backward(ctx, dout):
        return dout.expand(dout.shape[0], ctx.T, dout.shape[2]), None


def local_track_params(model) -> List[torch.nn.Parameter]:
    """Parameters whose gradients are per-shard partials under CP (summed over the group).  In paper
    semantics the attention's key / value projections are too (h2^T dpre over this shard's positions);
    the query projection's gradient comes from the all-reduced query gradient, i.e. already complete."""
    out = [model.local_embedding.weight, *model.pretraining_local_output.parameters()]
    for blk in model.proteinBERT_blocks:
        out += [*blk.local_narrow_conv_layer.parameters(), *blk.local_wide_conv_layer.parameters(),
                *blk.local_norm_1.parameters(), *blk.local_norm_2.parameters(), *blk.local_linear_layer.parameters()]
        if getattr(model, "semantics", "reference") == "paper":
            att = blk.global_attention_layer
            out += [p for p in (att.Wk, att.Wv) if isinstance(p, torch.nn.Parameter)]
    return out


def cp_reduce_grads(model, cp: CPShard, params: Optional[List[torch.nn.Parameter]] = None) -> None:
    """SUM the local-track parameters' gradients over the CP group (one coalesced all-reduce); the
    replicated parameters already hold the full gradient on every rank."""
    ps = [p for p in (params or local_track_params(model)) if p.grad is not None]
    if not ps:
        return
    flat = torch.cat([p.grad.reshape(-1) for p in ps])
    dist.all_reduce(flat, group=cp.group)
    o = 0
    for p in ps:
        n = p.grad.numel()
        p.grad.copy_(flat[o:o + n].view_as(p.grad))
        o += n


def cp_loss(model, cp: CPShard, X, Y, W):
    """This rank's fused loss under CP: ``(loss_for_backward, full_loss)`` -- backward the first (the
    rank's share of the CE + the replicated BCE), report the second (the group-wide loss, one
    all-reduce of the CE share)."""
    from ..ops.fused_model import fused_pretrain_loss
    total, l_local, l_global = fused_pretrain_loss(model, X, Y, W, return_parts=True, cp=cp)
    ce = l_local.detach().clone()
    dist.all_reduce(ce, group=cp.group)
    return total, ce + l_global.detach()


__all__ = ["CPShard", "cp_reduce_grads", "cp_loss", "local_track_params"]
