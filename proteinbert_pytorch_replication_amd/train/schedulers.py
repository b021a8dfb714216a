"""Learning-rate schedule: linear warmup, then ReduceLROnPlateau.

Reference (``ProteinBERT/utils.py:256-264,319``) builds
``SequentialLR([LambdaLR(step / warmup), ReduceLROnPlateau], [warmup])``,
which raises ``ValueError`` on torch 2.10 and, on older torch, never feeds
the plateau phase a metric.  This scheduler does what was
intended: ``warmup_duration`` steps of ``lr = base * step / warmup`` (the
reference lambda, which starts at 0 — quirk Q8 kept), then plateau
reduction driven by the training loss.

Checkpoints keep the reference's three keys: ``scheduler_state_dict``
(plateau), ``warmup_scheduler_state_dict`` (warmup) and
``full_scheduler_state_dict`` (this combined object).
"""
from __future__ import annotations

import warnings
from typing import Any, Dict, Optional

import torch
from torch.optim.lr_scheduler import LambdaLR, ReduceLROnPlateau


class _Warmup:
    def __init__(self, warmup_duration: int):
        self.warmup_duration = max(1, int(warmup_duration))

    def __call__(self, step: int) -> float:
        return float(step / self.warmup_duration)


class WarmupThenPlateau:
    def __init__(self, optimizer: torch.optim.Optimizer, warmup_duration: int = 10000, patience: int = 25,
                 factor: float = 0.1, mode: str = "min"):
        self.optimizer = optimizer
        self.warmup_duration = int(warmup_duration)
        self.warmup = LambdaLR(optimizer, lr_lambda=_Warmup(warmup_duration))
        self.plateau = ReduceLROnPlateau(optimizer, mode=mode, patience=patience, factor=factor)
        self.last_step = 0

    @property
    def in_warmup(self) -> bool:
        return self.last_step < self.warmup_duration

    def step(self, metric: Optional[float] = None) -> None:
        self.last_step += 1
        if self.last_step <= self.warmup_duration:
            with warnings.catch_warnings():
                warnings.simplefilter("ignore", UserWarning)  # step-order warning: we own the order
                self.warmup.step()
        elif metric is not None:
            self.plateau.step(metric)

    def get_last_lr(self):
        return [g["lr"] for g in self.optimizer.param_groups]

    def state_dict(self) -> Dict[str, Any]:
        return {"last_step": self.last_step, "warmup_duration": self.warmup_duration,
                "lrs": self.get_last_lr()}

    def load_state_dict(self, state: Dict[str, Any]) -> None:
        self.last_step = int(state["last_step"])
        for g, lr in zip(self.optimizer.param_groups, state.get("lrs", [])):
            g["lr"] = lr

    def state_dicts(self) -> Dict[str, Dict[str, Any]]:
        return {"scheduler_state_dict": self.plateau.state_dict(),
                "warmup_scheduler_state_dict": self.warmup.state_dict(),
                "full_scheduler_state_dict": self.state_dict()}

    def load_state_dicts(self, ckpt: Dict[str, Any]) -> None:
        if "scheduler_state_dict" in ckpt:
            self.plateau.load_state_dict(ckpt["scheduler_state_dict"])
        if "warmup_scheduler_state_dict" in ckpt:
            w = dict(ckpt["warmup_scheduler_state_dict"])
            w.setdefault("lr_lambdas", [None])
            self.warmup.load_state_dict(w)
        full = ckpt.get("full_scheduler_state_dict")
        if full and "last_step" in full:
            self.load_state_dict(full)
        elif full and "last_epoch" in full:  # reference SequentialLR state
            self.last_step = int(full["last_epoch"])
