"""ProteinBERT: dual-track (local per-residue / global per-protein) encoder.

Reference: ``ProteinBERT/modules.py`` (``GlobalAttentionHead`` :21-60,
``GlobalAttention`` :63-92, ``ProteinBERTBlock`` :95-231, ``ProteinBERT``
:234-304).  Same constructor signature, same ``forward(dict) -> (probs_local,
probs_global)`` API and the same 133-key ``state_dict`` (names, shapes and
``[out, in, (k)]`` layouts), so reference checkpoints load with
``strict=True`` both ways.

What differs is the inside:

* activations are channels-last ``[B, L, C]`` end to end (the reference
  permutes between ``[B, C, L]`` and ``[B, L, C]`` inside every block);
* on a GPU the block runs through fused CDNA4 HIP kernels (``ops/``):
  dual-dilation implicit-GEMM conv with fused GELU/residual/broadcast
  epilogue, two-phase whole-sequence LayerNorm, fused local MLP, fused
  attention pool, fused heads + loss; ``backend="torch"`` is the eager oracle;
* attention-head weights are real tensors of the module (stacked
  ``[H, ...]``), moved by ``.to()``; in reference semantics they are
  non-persistent buffers (the reference keeps them in a plain list, so they
  are neither trained nor checkpointed, ``modules.py:73-81``) and are saved
  by the trainer under ``extra_state``.

Semantics (``semantics=``):

``reference`` (default) reproduces the reference's math exactly, quirks
included: the attention softmax runs over the key axis whose
rows are identical, so every head reduces *exactly* (P == 1/K in fp32) to
``(1/K) * sum_l GELU(h Wv)``; the local head's ``nn.Softmax()`` runs over
the batch axis; LayerNorm normalises over ``(L, C)`` with ``[L, C]`` affine.

``paper`` is the published model: per-head single-query attention with the
softmax over sequence positions, local softmax over the vocabulary and
per-position LayerNorm over channels (``[C]`` affine; not
checkpoint-compatible with the reference).
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

_DEFAULT_DEVICE = "cpu"


def _gelu(x: torch.Tensor) -> torch.Tensor:
    return F.gelu(x)  # exact erf GELU == nn.GELU() default


class GlobalAttentionHead(nn.Module):
    """One local -> global attention head as a standalone module, reference API
    (``modules.py:21-60``): ``Wv_parameter [C, vd]``, ``Wk_parameter [C, K]``, ``Wq_parameter [G, K]``
    (``randn`` init), ``forward({"local": [B, L, C], "global": [B, G]}) -> [B, K, vd]``.

    ``semantics="reference"``: the reference's softmax runs over the K identical query rows, so every
    output row is exactly ``(1/K) sum_l GELU(h Wv)`` -- computed in that closed form (Q and K never
    influence the result); :meth:`forward_faithful` is the literal computation.  ``"paper"``: one
    query per head, softmax over positions, the ``[B, vd]`` result repeated over the K rows.
    :class:`GlobalAttention` holds the heads of a block stacked for the fused kernels.
    """

    def __init__(self, local_dim: int, global_dim: int, value_dim: int, key_dim: int, device=None,
                 semantics: str = "reference"):
        super().__init__()
        device = device or _DEFAULT_DEVICE
        self.key_dim, self.global_dim, self.semantics = key_dim, global_dim, semantics
        self.Wv_parameter = nn.Parameter(torch.randn(local_dim, value_dim, device=device))
        self.Wk_parameter = nn.Parameter(torch.randn(local_dim, key_dim, device=device))
        self.Wq_parameter = nn.Parameter(torch.randn(global_dim, key_dim, device=device))

    def forward_faithful(self, x: Dict[str, torch.Tensor]) -> torch.Tensor:
        K = self.key_dim
        q = torch.tanh(torch.matmul(x["global"].unsqueeze(1).expand(-1, K, -1), self.Wq_parameter))
        k = torch.tanh(torch.matmul(x["local"], self.Wk_parameter))
        v = _gelu(torch.matmul(x["local"], self.Wv_parameter))
        return torch.matmul(torch.softmax(torch.matmul(q, k.transpose(1, 2)) / math.sqrt(K), dim=1), v)

    def forward(self, x: Dict[str, torch.Tensor]) -> torch.Tensor:
        h, K = x["local"], self.key_dim
        v = _gelu(torch.matmul(h, self.Wv_parameter))                                   # [B, L, vd]
        if self.semantics == "paper":
            q = torch.tanh(torch.matmul(x["global"], self.Wq_parameter))               # [B, K]
            k = torch.tanh(torch.matmul(h, self.Wk_parameter))                         # [B, L, K]
            p = torch.softmax(torch.einsum("bk,blk->bl", q, k) / math.sqrt(K), dim=-1)
            o = torch.einsum("bl,blv->bv", p, v)
        else:
            o = v.sum(dim=1) / K
        return o.unsqueeze(1).expand(-1, K, -1)


class _HeadView:
    """Read/write view of one stacked attention head, named like the reference
    ``GlobalAttentionHead`` attributes (``modules.py:36-47``)."""

    def __init__(self, owner: "GlobalAttention", j: int):
        self._o, self._j = owner, j

    @property
    def Wv_parameter(self) -> torch.Tensor:
        return self._o.Wv[self._j]

    @property
    def Wk_parameter(self) -> torch.Tensor:
        return self._o.Wk[self._j]

    @property
    def Wq_parameter(self) -> torch.Tensor:
        return self._o.Wq[self._j]


class GlobalAttention(nn.Module):
    """Local -> global attention over ``num_heads`` heads (reference ``modules.py:21-92``).

    Heads are stacked: ``Wv [H, C, vd]``, ``Wk [H, C, K]``, ``Wq [H, G, K]``.
    ``W_parameter [K]`` is registered exactly as in the reference.
    """

    def __init__(self, num_heads: int, local_dim: int, global_dim: int, value_dim: int, key_dim: int,
                 device=None, semantics: str = "reference", train_heads: Optional[bool] = None):
        super().__init__()
        device = device or _DEFAULT_DEVICE
        self.num_heads, self.local_dim, self.global_dim = num_heads, local_dim, global_dim
        self.value_dim, self.key_dim = value_dim, key_dim
        self.semantics = semantics
        if train_heads is None:
            train_heads = semantics == "paper"
        self.train_heads = train_heads
        Wv = torch.randn(num_heads, local_dim, value_dim, device=device)
        Wk = torch.randn(num_heads, local_dim, key_dim, device=device)
        Wq = torch.randn(num_heads, global_dim, key_dim, device=device)
        if train_heads:
            self.Wv, self.Wk, self.Wq = nn.Parameter(Wv), nn.Parameter(Wk), nn.Parameter(Wq)
        else:
            # reference: plain-list heads -> not in state_dict, not optimised
            self.register_buffer("Wv", Wv, persistent=False)
            self.register_buffer("Wk", Wk, persistent=False)
            self.register_buffer("Wq", Wq, persistent=False)
        self.W_parameter = nn.Parameter(torch.randn(key_dim, device=device))

    @property
    def global_attention_heads(self):
        return [_HeadView(self, j) for j in range(self.num_heads)]

    def heads_state(self) -> Dict[str, torch.Tensor]:
        return {"Wv": self.Wv.detach().clone(), "Wk": self.Wk.detach().clone(),
                "Wq": self.Wq.detach().clone()}

    def load_heads_state(self, state: Dict[str, torch.Tensor]) -> None:
        with torch.no_grad():
            for k in ("Wv", "Wk", "Wq"):
                getattr(self, k).copy_(state[k])

    def value_weight_cat(self) -> torch.Tensor:
        """``[C, H*vd]`` = heads' Wv concatenated on the output axis (cat order of ``modules.py:92``)."""
        return self.Wv.permute(1, 0, 2).reshape(self.local_dim, self.num_heads * self.value_dim)

    # --- torch (oracle) paths -------------------------------------------------
    def forward_faithful(self, h: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
        """Literal reference computation (Q/K/softmax over dim=1), channels-last input."""
        outs = []
        K = self.key_dim
        for j in range(self.num_heads):
            q = torch.tanh(torch.matmul(g.unsqueeze(1).expand(-1, K, -1), self.Wq[j]))   # [B,K,K]
            k = torch.tanh(torch.matmul(h, self.Wk[j]))                                 # [B,L,K]
            v = _gelu(torch.matmul(h, self.Wv[j]))                                      # [B,L,vd]
            s = torch.matmul(q, k.transpose(1, 2)) / torch.sqrt(torch.tensor(float(K)))
            outs.append(torch.matmul(torch.softmax(s, dim=1), v))                       # [B,K,vd]
        return torch.matmul(self.W_parameter, torch.cat(outs, dim=2))                   # [B,G]

    def forward_closed_form(self, h: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
        """Exact closed form of the reference attention: (sum W / K) * sum_l GELU(h Wv)."""
        v = _gelu(torch.matmul(h, self.value_weight_cat().to(h.dtype)))                # [B,L,G]
        scale = self.W_parameter.sum() / self.key_dim
        return v.float().sum(dim=1) * scale

    def forward_paper(self, h: torch.Tensor, g: torch.Tensor,
                      mask: Optional[torch.Tensor] = None, use_kernel: bool = True) -> torch.Tensor:
        """Per-head single query from the global track, softmax over positions.

        bf16 on a GPU runs the split-L HIP core (``ops/paper_attention.py``); ``use_kernel=False``
        (or any other dtype/device) is the torch oracle below.
        """
        if use_kernel:
            from ..ops import paper_attention as pa
            if pa.kernel_supported(h, self.key_dim, self.value_dim):
                return pa.paper_attention(h, g, self.Wq, self.Wk, self.Wv, mask)
        q = torch.tanh(torch.einsum("bg,hgk->bhk", g, self.Wq.to(g.dtype)))            # [B,H,K]
        k = torch.tanh(torch.einsum("blc,hck->bhlk", h, self.Wk.to(h.dtype)))          # [B,H,L,K]
        v = _gelu(torch.einsum("blc,hcv->bhlv", h, self.Wv.to(h.dtype)))               # [B,H,L,vd]
        s = torch.einsum("bhk,bhlk->bhl", q.to(k.dtype), k).float() / math.sqrt(self.key_dim)
        if mask is not None:
            s = s.masked_fill(~mask.unsqueeze(1), float("-inf"))
        p = torch.softmax(s, dim=-1)
        o = torch.einsum("bhl,bhlv->bhv", p.to(v.dtype), v)
        return o.reshape(o.shape[0], -1).float()

    def forward(self, x: Dict[str, torch.Tensor]) -> torch.Tensor:
        """Reference-shaped call: ``x["local"]`` is ``[B, L, C]`` (as in ``modules.py:219``)."""
        if self.semantics == "paper":
            return self.forward_paper(x["local"], x["global"])
        return self.forward_closed_form(x["local"], x["global"])


class ProteinBERTBlock(nn.Module):
    """One dual-track block (reference ``modules.py:95-231``); channels-last I/O ``[B, L, C]``."""

    def __init__(self, sequences_length, local_dim: int, global_dim: int, num_heads: int, key_dim: int,
                 conv_kernel_size: int = 9, wide_conv_dilation: int = 5, device=None,
                 semantics: str = "reference"):
        super().__init__()
        assert global_dim % num_heads == 0, \
            f"Global_dim must be divisible by num_heads. Global_dim: {global_dim}. Num_heads: {num_heads}"
        device = device or _DEFAULT_DEVICE
        self.sequences_length, self.local_dim, self.global_dim = sequences_length, local_dim, global_dim
        self.conv_kernel_size, self.wide_conv_dilation = conv_kernel_size, wide_conv_dilation
        self.semantics = semantics
        self.global_attention_layer = GlobalAttention(num_heads, local_dim, global_dim,
                                                      int(global_dim / num_heads), key_dim, device, semantics)
        conv = lambda d: nn.Sequential(nn.Conv1d(local_dim, local_dim, conv_kernel_size, stride=1, dilation=d,  # noqa: E731
                                                 padding="same", device=device), nn.GELU())
        self.local_narrow_conv_layer = conv(1)
        self.local_wide_conv_layer = conv(wide_conv_dilation)
        ln_shape = (sequences_length, local_dim) if semantics == "reference" else (local_dim,)
        self.local_norm_1 = nn.LayerNorm(ln_shape, device=device)
        self.local_linear_layer = nn.Sequential(nn.Linear(local_dim, local_dim, device=device), nn.GELU())
        self.local_norm_2 = nn.LayerNorm(ln_shape, device=device)
        self.global_to_local_linear_layer = nn.Sequential(nn.Linear(global_dim, local_dim, device=device),
                                                          nn.GELU())
        self.global_linear_layer_1 = nn.Sequential(nn.Linear(global_dim, global_dim, device=device), nn.GELU())
        self.global_norm_1 = nn.LayerNorm(global_dim, device=device)
        self.global_linear_layer_2 = nn.Sequential(nn.Linear(global_dim, global_dim, device=device), nn.GELU())
        self.global_norm_2 = nn.LayerNorm(global_dim, device=device)

    # -- torch (oracle) path ----------------------------------------------------
    def _conv(self, seq: nn.Sequential, h: torch.Tensor) -> torch.Tensor:
        conv: nn.Conv1d = seq[0]
        w = conv.weight.to(h.dtype)
        b = conv.bias.to(h.dtype)
        return _gelu(F.conv1d(h.transpose(1, 2), w, b, padding="same",
                              dilation=conv.dilation).transpose(1, 2))

    def _local_norm(self, ln: nn.LayerNorm, x: torch.Tensor) -> torch.Tensor:
        if self.semantics == "reference" and x.shape[1] != ln.normalized_shape[0]:
            # variable-length model (ProteinBERT(variable_length=True)): the [L_max, C] affine is sliced
            # to the batch's L; the statistics span the batch's L x C elements
            L = x.shape[1]
            return F.layer_norm(x.float(), (L, ln.normalized_shape[1]), ln.weight[:L], ln.bias[:L],
                                ln.eps).to(x.dtype)
        return F.layer_norm(x.float(), ln.normalized_shape, ln.weight, ln.bias, ln.eps).to(x.dtype)

    def forward_torch(self, h: torch.Tensor, g: torch.Tensor, mask: Optional[torch.Tensor] = None,
                      faithful_attention: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
        lin = lambda seq, x: _gelu(F.linear(x, seq[0].weight.to(x.dtype), seq[0].bias.to(x.dtype)))  # noqa: E731
        n = self._conv(self.local_narrow_conv_layer, h)
        w = self._conv(self.local_wide_conv_layer, h)
        gb = lin(self.global_to_local_linear_layer, g.to(h.dtype))
        s1 = h + n + w + gb.unsqueeze(1)
        h1 = self._local_norm(self.local_norm_1, s1)
        s2 = h1 + lin(self.local_linear_layer, h1)
        h2 = self._local_norm(self.local_norm_2, s2)
        att = self.global_attention_layer
        if self.semantics == "paper":
            ga = att.forward_paper(h2, g, mask)
        elif faithful_attention:
            ga = att.forward_faithful(h2.float(), g.float())
        else:
            ga = att.forward_closed_form(h2, g)
        gf = g.float()
        g1 = F.layer_norm(gf + lin(self.global_linear_layer_1, gf) + ga, self.global_norm_1.normalized_shape,
                          self.global_norm_1.weight, self.global_norm_1.bias, self.global_norm_1.eps)
        g2 = F.layer_norm(g1 + lin(self.global_linear_layer_2, g1), self.global_norm_2.normalized_shape,
                          self.global_norm_2.weight, self.global_norm_2.bias, self.global_norm_2.eps)
        return h2, g2

    def forward(self, x: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        h, g = self.forward_torch(x["local"], x["global"])
        return {"local": h, "global": g}


class ProteinBERT(nn.Module):
    """Reference-compatible ProteinBERT (``modules.py:234-304``).

    ``backend``: ``"auto"`` (HIP kernels when on a GPU, else torch), ``"hip"``
    or ``"torch"``.  ``compute_dtype``: dtype of activations on the fast path
    (bf16 by default on GPU; parameters stay fp32 masters).

    ``variable_length``: the reference ties its ``LayerNorm((L, C))`` affine to one length
    (``modules.py:148-151,161-164``; any other L raises).  With ``variable_length=True`` the affine is
    stored at ``L_max = sequences_length`` and a batch of length ``L <= L_max`` uses rows ``[:L]``
    (statistics over its own L x C elements), so one model trains on the paper's mixed lengths
    (128 / 512 / 1024).  The state dict keeps the reference key set with ``[L_max, C]`` shapes; a
    reference model loads it only at ``sequences_length == L_max``.
    """

    def __init__(self, sequences_length: int, num_annotations: int, local_dim: int, global_dim: int,
                 key_dim: int, num_heads: int, num_blocks: int, conv_kernel_size: int = 9,
                 wide_conv_dilation: int = 5, vocab_size: int = 26, device=None,
                 semantics: str = "reference", backend: str = "auto", variable_length: bool = False):
        super().__init__()
        if semantics not in ("reference", "paper"):
            raise ValueError(f"semantics must be 'reference' or 'paper', got {semantics!r}")
        device = device or _DEFAULT_DEVICE
        self.config = dict(sequences_length=sequences_length, num_annotations=num_annotations,
                           local_dim=local_dim, global_dim=global_dim, key_dim=key_dim, num_heads=num_heads,
                           num_blocks=num_blocks, conv_kernel_size=conv_kernel_size,
                           wide_conv_dilation=wide_conv_dilation, vocab_size=vocab_size, semantics=semantics,
                           variable_length=variable_length)
        self.semantics = semantics
        self.variable_length = variable_length
        self.sequences_length = sequences_length
        self.backend = backend
        self.local_embedding = nn.Embedding(vocab_size, local_dim, device=device)
        self.global_linear_layer = nn.Sequential(nn.Linear(num_annotations, global_dim, device=device), nn.GELU())
        self.proteinBERT_blocks = nn.Sequential(*[
            ProteinBERTBlock(sequences_length, local_dim, global_dim, num_heads, key_dim, conv_kernel_size,
                             wide_conv_dilation, device, semantics) for _ in range(num_blocks)])
        self.pretraining_local_output = nn.Sequential(nn.Linear(local_dim, vocab_size, device=device),
                                                      nn.Softmax(dim=0 if semantics == "reference" else -1))
        self.pretraining_global_output = nn.Sequential(nn.Linear(global_dim, num_annotations, device=device),
                                                       nn.Sigmoid())
        self._fast = None  # lazily-built HIP executor (ops.fused_model.FusedProteinBERT)

    # ------------------------------------------------------------------------
    def resolved_backend(self, device: torch.device) -> str:
        # deterministic mode routes configurations without fixed-order HIP kernels (paper semantics,
        # general global-track shapes) to the PyTorch path, judged on this model's own config (so a
        # checkpoint loaded with another preset's flags is routed by what it is)
        from ..utils import determinism
        backend = determinism.backend_for(self.backend, self.config)
        if backend == "auto":
            if device.type != "cuda":
                return "torch"
            from ..ops.fused_model import hip_supported
            return "hip" if hip_supported(self)[0] else "torch"
        return backend

    def attention_heads_state(self) -> Dict[str, Dict[str, torch.Tensor]]:
        return {str(i): b.global_attention_layer.heads_state() for i, b in enumerate(self.proteinBERT_blocks)}

    def load_attention_heads_state(self, state: Dict[str, Dict[str, torch.Tensor]]) -> None:
        for i, b in enumerate(self.proteinBERT_blocks):
            b.global_attention_layer.load_heads_state(state[str(i)])

    # ------------------------------------------------------------------------
    def check_length(self, L: int) -> None:
        """Reference semantics: the LayerNorm affine fixes L (exactly ``sequences_length``, or at most
        it for a ``variable_length`` model); paper semantics (per-position LN) takes any L."""
        if self.semantics != "reference":
            return
        if L > self.sequences_length or (L != self.sequences_length and not self.variable_length):
            raise RuntimeError(f"input length {L} does not match the model's LayerNorm((L, C)) length "
                               f"{self.sequences_length}" + ("" if self.variable_length else
                                                             " (build with variable_length=True for L < L_max)"))

    def encode_torch(self, tokens: torch.Tensor, annotations: torch.Tensor,
                     compute_dtype: Optional[torch.dtype] = None,
                     faithful_attention: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
        self.check_length(tokens.shape[1])
        dt = compute_dtype or torch.float32
        h = self.local_embedding.weight.to(dt)[tokens]                       # [B,L,C]
        lin = self.global_linear_layer[0]
        g = _gelu(F.linear(annotations.to(dt), lin.weight.to(dt), lin.bias.to(dt))).float()
        mask = tokens != 0 if self.semantics == "paper" else None
        for blk in self.proteinBERT_blocks:
            h, g = blk.forward_torch(h, g, mask, faithful_attention)
        return h, g

    def heads_torch(self, h: torch.Tensor, g: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        lo = self.pretraining_local_output[0]
        logits_l = F.linear(h.float(), lo.weight, lo.bias)                      # [B,L,V]
        if self.semantics == "reference":
            from ..parallel.batch_softmax import softmax_over_batch
            probs_l = softmax_over_batch(logits_l)     # this rank's batch, or the DP group's (dp_batch_softmax)
        else:
            probs_l = torch.softmax(logits_l, dim=-1)
        go = self.pretraining_global_output[0]
        probs_g = torch.sigmoid(F.linear(g.float(), go.weight, go.bias))
        return probs_l, probs_g

    def forward(self, x: Dict[str, torch.Tensor]) -> Tuple[torch.Tensor, torch.Tensor]:
        tokens, ann = x["local"], x["global"]
        if self.resolved_backend(tokens.device) == "hip":
            from ..ops.fused_model import fused_forward
            return fused_forward(self, tokens, ann)
        h, g = self.encode_torch(tokens, ann)
        return self.heads_torch(h, g)


def build_model(cfg, device=None, backend: str = "auto") -> ProteinBERT:
    """Construct from a :class:`~..config.ModelConfig`."""
    kw = cfg.kwargs() if hasattr(cfg, "kwargs") else dict(cfg)
    return ProteinBERT(device=device, backend=backend, **kw)
