"""Pretraining losses.

Reference (``ProteinBERT/utils.py:293-294``)::

    loss = mean(CE(probs_local.permute(0, 2, 1), y_local) * w_local)
         + mean(BCE(probs_global, y_global) * w_global)

with ``CE = nn.CrossEntropyLoss(reduction='none')`` applied to the model's
*probabilities* (a second softmax) and
``BCE = nn.BCELoss(reduction='none')`` (log clamped at -100).  Means run over
``B*L`` and ``B*A`` including zero-weight entries.  In ``paper`` semantics the
local term is the NLL of the predicted distribution instead.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F


def pretrain_loss_torch(probs_l: torch.Tensor, probs_g: torch.Tensor, Y: Dict[str, torch.Tensor],
                        W: Dict[str, torch.Tensor], semantics: str = "reference",
                        local_loss_fn=None, global_loss_fn=None,
                        return_parts: bool = False):
    y_l, y_g = Y["local"], Y["global"].float()
    if local_loss_fn is not None:
        ce = local_loss_fn(probs_l.permute(0, 2, 1), y_l)
    elif semantics == "reference":
        ce = F.cross_entropy(probs_l.permute(0, 2, 1).float(), y_l, reduction="none")
    else:
        ce = F.nll_loss(torch.log(probs_l.float().clamp_min(1e-30)).permute(0, 2, 1), y_l, reduction="none")
    if global_loss_fn is not None:
        bce = global_loss_fn(probs_g, y_g)
    else:
        bce = F.binary_cross_entropy(probs_g.float(), y_g, reduction="none")
    local = torch.mean(ce * W["local"])
    glob = torch.mean(bce * W["global"])
    if return_parts:
        return local + glob, local, glob
    return local + glob


def is_standard_loss_pair(local_loss_fn, global_loss_fn) -> bool:
    """True when the user passed the reference's loss modules (so the fused path is exact)."""
    ok_l = local_loss_fn is None or (isinstance(local_loss_fn, torch.nn.CrossEntropyLoss)
                                     and local_loss_fn.reduction == "none" and local_loss_fn.weight is None
                                     and local_loss_fn.ignore_index == -100
                                     and local_loss_fn.label_smoothing == 0.0)
    ok_g = global_loss_fn is None or (isinstance(global_loss_fn, torch.nn.BCELoss)
                                      and global_loss_fn.reduction == "none" and global_loss_fn.weight is None)
    return ok_l and ok_g
