"""Checkpoint / resume with the reference's file contract.

Reference (``ProteinBERT/utils.py:324-343``): every ``nb_iterations_checkpoint``
iterations ``torch.save`` of a 7-key dict to
``proteinbert_pretraining_checkpoint_{iter}.pt``, and a final whole-model pickle
``proteinbert_pretrained_model_{%m-%d-%Y_%H-%M-%S}.pt``.

Here:

* the 7 keys are written with the same names and meanings; the
  ``model_state_dict`` is strict-loadable by the reference ``ProteinBERT``;
* ``extra_state`` adds what the reference loses on resume:
  the attention-head weights (unregistered in the reference), RNG states,
  data cursor, world size, config;
* writes are atomic (tmp + rename), rank 0 only, optionally on a background
  thread;
* the "final model" file is a state-dict + config bundle (no pickled code),
  so it loads with ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import datetime
import logging
import os
import threading
from typing import Any, Dict, Optional

import torch

log = logging.getLogger("pbx.checkpoint")

REFERENCE_KEYS = ("current_batch_iteration", "model_state_dict", "optimizer_state_dict", "scheduler_state_dict",
                  "warmup_scheduler_state_dict", "full_scheduler_state_dict", "loss")


def checkpoint_name(iteration: int) -> str:
    return f"proteinbert_pretraining_checkpoint_{iteration}.pt"


def final_model_name(now: Optional[datetime.datetime] = None) -> str:
    now = now or datetime.datetime.now()
    return f"proteinbert_pretrained_model_{now.strftime('%m-%d-%Y_%H-%M-%S')}.pt"


def _to_cpu(obj: Any) -> Any:
    if isinstance(obj, torch.Tensor):
        return obj.detach().to("cpu", copy=True)
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


def rng_state(device: Optional[torch.device] = None) -> Dict[str, Any]:
    st = {"torch": torch.get_rng_state()}
    if device is not None and device.type == "cuda":
        st["cuda"] = torch.cuda.get_rng_state(device)
    return st


def set_rng_state(st: Dict[str, Any], device: Optional[torch.device] = None) -> None:
    if "torch" in st:
        torch.set_rng_state(st["torch"].cpu())
    if "cuda" in st and device is not None and device.type == "cuda":
        torch.cuda.set_rng_state(st["cuda"].cpu(), device)


def build_checkpoint(iteration: int, model, optimizer, scheduler, loss: float,
                     extra: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
    ckpt = {"current_batch_iteration": int(iteration),
            "model_state_dict": model.state_dict(),
            "optimizer_state_dict": optimizer.state_dict()}
    ckpt.update(scheduler.state_dicts())
    ckpt["loss"] = float(loss)
    extra = dict(extra or {})
    if hasattr(model, "attention_heads_state"):
        extra.setdefault("attention_heads", model.attention_heads_state())
    if hasattr(model, "config"):
        extra.setdefault("config", dict(model.config))
    ckpt["extra_state"] = extra
    return _to_cpu(ckpt)


def atomic_save(obj: Dict[str, Any], path: str) -> None:
    tmp = f"{path}.tmp.{os.getpid()}"
    torch.save(obj, tmp)
    os.replace(tmp, path)


class CheckpointWriter:
    """Rank-0 writer; ``async_save`` moves serialisation off the training thread
    (state is snapshot to CPU synchronously, so the step can continue)."""

    def __init__(self, save_path: str, async_save: bool = False, is_main: bool = True):
        self.save_path = save_path
        self.async_save = async_save
        self.is_main = is_main
        self._thread: Optional[threading.Thread] = None
        if is_main:
            os.makedirs(save_path, exist_ok=True)

    def save(self, ckpt: Dict[str, Any], name: str) -> str:
        path = os.path.join(self.save_path, name)
        if not self.is_main:
            return path
        self.wait()
        if self.async_save:
            self._thread = threading.Thread(target=atomic_save, args=(ckpt, path), daemon=True)
            self._thread.start()
        else:
            atomic_save(ckpt, path)
        log.info("Checkpoint saved to %s", path)
        return path

    def wait(self) -> None:
        if self._thread is not None:
            self._thread.join()
            self._thread = None


def load_checkpoint(path: str, map_location="cpu") -> Dict[str, Any]:
    """Safe load (no code execution): ``weights_only=True``."""
    return torch.load(path, map_location=map_location, weights_only=True)


def latest_checkpoint(save_path: str) -> Optional[str]:
    best, best_it = None, -1
    if not os.path.isdir(save_path):
        return None
    for f in os.listdir(save_path):
        if f.startswith("proteinbert_pretraining_checkpoint_") and f.endswith(".pt"):
            try:
                it = int(f[len("proteinbert_pretraining_checkpoint_"):-3])
            except ValueError:
                continue
            if it > best_it:
                best, best_it = os.path.join(save_path, f), it
    return best


def load_reference_checkpoint(model, ckpt: Dict[str, Any], head_seed: int = 0) -> None:
    """Load a reference-produced checkpoint dict.  The reference never saves its
    attention-head weights; when ``extra_state`` lacks them they are re-drawn
    from a seeded ``randn`` (deterministic, unlike the reference) and a warning
    is logged."""
    model.load_state_dict(ckpt["model_state_dict"], strict=True)
    heads = ckpt.get("extra_state", {}).get("attention_heads")
    if heads is not None:
        model.load_attention_heads_state(heads)
        return
    log.warning("checkpoint has no attention-head weights (reference layout); re-initialising them "
                "with seed %d", head_seed)
    g = torch.Generator().manual_seed(head_seed)
    for blk in model.proteinBERT_blocks:
        att = blk.global_attention_layer
        with torch.no_grad():
            for name in ("Wv", "Wk", "Wq"):
                t = getattr(att, name)
                t.copy_(torch.randn(t.shape, generator=g).to(t.device))


def save_final_model(model, save_path: str, is_main: bool = True) -> str:
    path = os.path.join(save_path, final_model_name())
    if is_main:
        atomic_save(_to_cpu({"config": dict(getattr(model, "config", {})),
                             "model_state_dict": model.state_dict(),
                             "extra_state": {"attention_heads": model.attention_heads_state()}}), path)
        log.info("Whole model saved to %s", path)
    return path


def load_model(path: str, device=None, backend: str = "auto"):
    from ..models import ProteinBERT
    blob = load_checkpoint(path)
    cfg = dict(blob["config"])
    model = ProteinBERT(device=device, backend=backend, **cfg)
    load_reference_checkpoint(model, blob)
    return model
