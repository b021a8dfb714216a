"""Fine-tuning heads on the ProteinBERT encoder (BASELINE cfg 5).

The reference ships generic ``train_step``/``test_step`` loops (``ProteinBERT/utils.py:110-217``)
that call ``model(X)`` and apply ``loss_fn(logits, y)`` and ``softmax(logits, dim=1)``; it has no
fine-tuning model.  These heads follow that contract: the class axis is dim 1.

* :class:`ProteinBERTForTokenClassification` - per-residue head (e.g. 3- or 8-state secondary
  structure): logits ``[B, n_classes, L]``.
* :class:`ProteinBERTForSequenceClassification` - per-protein head on the global track:
  logits ``[B, n_classes]``.

``freeze_encoder=True`` runs the encoder under ``torch.no_grad`` (no activations are kept, so a
frozen-encoder step costs one forward of the fused HIP encoder plus the tiny head); with
``freeze_encoder=False`` gradients flow through the fused HIP backward as in pretraining.
Inputs: a token tensor ``[B, L]`` (annotations default to zeros, i.e. "no GO prior") or the
pretraining dict ``{"local": tokens, "global": annotations}``.
"""
from __future__ import annotations

from typing import Dict, Tuple, Union

import torch
import torch.nn as nn
import torch.nn.functional as F

from .proteinbert import ProteinBERT

Inputs = Union[torch.Tensor, Dict[str, torch.Tensor]]


def _split_inputs(model: ProteinBERT, x: Inputs) -> Tuple[torch.Tensor, torch.Tensor]:
    if isinstance(x, dict):
        return x["local"], x["global"]
    A = model.config["num_annotations"]
    return x, torch.zeros((x.shape[0], A), dtype=torch.float32, device=x.device)


def encode(model: ProteinBERT, tokens: torch.Tensor, ann: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Encoder output ``h [B, L, C]``, ``g [B, G]`` on the model's backend (fused HIP on a GPU)."""
    if model.resolved_backend(tokens.device) == "hip":
        from ..ops.fused_model import fused_encode
        return fused_encode(model, tokens, ann.float())
    return model.encode_torch(tokens, ann.float())


class _FinetuneBase(nn.Module):
    def __init__(self, encoder: ProteinBERT, freeze_encoder: bool = True):
        super().__init__()
        self.encoder = encoder
        self.freeze_encoder = freeze_encoder
        if freeze_encoder:
            for p in encoder.parameters():
                p.requires_grad_(False)

    def _encode(self, x: Inputs) -> Tuple[torch.Tensor, torch.Tensor]:
        tokens, ann = _split_inputs(self.encoder, x)
        if self.freeze_encoder:
            with torch.no_grad():
                h, g = encode(self.encoder, tokens, ann)
            return h.detach(), g.detach()
        return encode(self.encoder, tokens, ann)

    def train(self, mode: bool = True):
        super().train(mode)
        if self.freeze_encoder:
            self.encoder.eval()
        return self


class ProteinBERTForTokenClassification(_FinetuneBase):
    def __init__(self, encoder: ProteinBERT, n_classes: int = 8, freeze_encoder: bool = True,
                 use_global: bool = True, dropout: float = 0.0):
        super().__init__(encoder, freeze_encoder)
        C, G = encoder.config["local_dim"], encoder.config["global_dim"]
        dev = encoder.local_embedding.weight.device
        self.use_global = use_global
        self.n_classes = n_classes
        self.dropout = nn.Dropout(dropout) if dropout > 0 else nn.Identity()
        self.head = nn.Linear(C, n_classes, device=dev)
        # per-residue logits = W_l h + (W_g g) broadcast over L  ==  Linear(concat(h, g))
        self.global_head = nn.Linear(G, n_classes, bias=False, device=dev) if use_global else None

    def forward(self, x: Inputs) -> torch.Tensor:
        h, g = self._encode(x)
        from ..ops import finetune_head
        if finetune_head.supported(h, self.n_classes) and isinstance(self.dropout, nn.Identity):
            # fp32-accurate split-weight bf16 GEMMs on the encoder output + streaming weight-gradient
            # kernel (ops/finetune_head.py)
            logits = finetune_head.TokenHeadFn.apply(h, self.head.weight, self.head.bias)
        else:
            logits = F.linear(self.dropout(h.float()), self.head.weight, self.head.bias)    # [B, L, K]
        if self.global_head is not None:
            logits = logits + self.global_head(g.float()).unsqueeze(1)
        return logits.permute(0, 2, 1)                                                   # [B, K, L]


class ProteinBERTForSequenceClassification(_FinetuneBase):
    def __init__(self, encoder: ProteinBERT, n_classes: int = 2, freeze_encoder: bool = True,
                 dropout: float = 0.0):
        super().__init__(encoder, freeze_encoder)
        G = encoder.config["global_dim"]
        dev = encoder.local_embedding.weight.device
        self.dropout = nn.Dropout(dropout) if dropout > 0 else nn.Identity()
        self.head = nn.Linear(G, n_classes, device=dev)

    def forward(self, x: Inputs) -> torch.Tensor:
        _, g = self._encode(x)
        return self.head(self.dropout(g.float()))
