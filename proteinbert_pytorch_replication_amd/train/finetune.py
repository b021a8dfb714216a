"""Fine-tuning loops (reference ``train_step`` / ``test_step``, ``ProteinBERT/utils.py:110-217``, T2/T3).

Same signatures and return values as the reference - ``(mean_loss, {metric_name: mean_value})`` per
epoch, metrics called as ``metric(softmax(logits, dim=1), y)`` - with these MI355X-side changes:

* no host sync per batch: loss and metric sums accumulate on the device and are read once at the
  end of the epoch (the reference calls ``loss.item()`` and ``.numpy()`` every batch);
* gradient clipping uses the fused arena grad-norm kernel when the optimizer is
  :class:`.optim.FusedAdam`, else ``torch.nn.utils.clip_grad_norm_``;
* ``X`` may be a tensor or the pretraining-style dict; ``(X, y)`` batches go to ``device`` with
  ``non_blocking`` copies;
* under data parallelism (``ddp`` given) gradients are all-reduced through the bucketed RCCL
  reducer before the optimizer step and the epoch means are averaged over ranks.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from ..parallel import dist as pdist
from .optim import FusedAdam


def _to(x, device):
    if isinstance(x, dict):
        return {k: v.to(device, non_blocking=True) for k, v in x.items()}
    return x.to(device, non_blocking=True)


def _metric_value(v) -> torch.Tensor:
    if isinstance(v, torch.Tensor):
        return v.detach().float().reshape(())
    return torch.tensor(float(v))


def _default_device():
    return "cuda" if torch.cuda.is_available() else "cpu"


def train_step(model: torch.nn.Module, dataloader, loss_fn: torch.nn.Module, optimizer: torch.optim.Optimizer,
               metrics: Dict[str, Callable], gradient_clipping: bool = True, gradient_clipping_thresh: float = 1,
               device=None, ddp=None) -> Tuple[float, Dict[str, float]]:
    device = torch.device(device or _default_device())
    model.train()
    loss_sum = torch.zeros((), dtype=torch.float32, device=device)
    met_sum = {k: torch.zeros((), dtype=torch.float32, device=device) for k in metrics}
    n = 0
    fused = isinstance(optimizer, FusedAdam)
    params = [p for p in model.parameters() if p.requires_grad]
    for X, y in dataloader:
        X, y = _to(X, device), _to(y, device)
        logits = model(X)
        loss = loss_fn(logits, y)
        loss_sum += loss.detach().float()
        optimizer.zero_grad()
        loss.backward()
        if ddp is not None:
            ddp.finish(average=not fused)
        if gradient_clipping:
            if fused:
                optimizer.clip_grad_norm_(gradient_clipping_thresh)
            else:
                torch.nn.utils.clip_grad_norm_(params, gradient_clipping_thresh)
        optimizer.step()
        if metrics:
            with torch.no_grad():
                preds = torch.softmax(logits.detach().float(), dim=1)
                for k, m in metrics.items():
                    met_sum[k] += _metric_value(m(preds, y)).to(device)
        n += 1
    return _finish(loss_sum, met_sum, n, ddp is not None)


def test_step(model: torch.nn.Module, dataloader, loss_fn: torch.nn.Module, metrics: Dict[str, Callable],
              device=None, distributed: bool = False) -> Tuple[float, Dict[str, float]]:
    device = torch.device(device or _default_device())
    model.eval()
    loss_sum = torch.zeros((), dtype=torch.float32, device=device)
    met_sum = {k: torch.zeros((), dtype=torch.float32, device=device) for k in metrics}
    n = 0
    with torch.inference_mode():
        for X, y in dataloader:
            X, y = _to(X, device), _to(y, device)
            logits = model(X)
            loss_sum += loss_fn(logits, y).float()
            preds = torch.softmax(logits.float(), dim=1)
            for k, m in metrics.items():
                met_sum[k] += _metric_value(m(preds, y)).to(device)
            n += 1
    return _finish(loss_sum, met_sum, n, distributed)


def _finish(loss_sum, met_sum, n, distributed) -> Tuple[float, Dict[str, float]]:
    vals = torch.stack([loss_sum] + [met_sum[k] for k in met_sum]) / max(1, n)
    if distributed:
        pdist.all_reduce_mean_(vals)
    vals = vals.cpu().tolist()
    return vals[0], {k: v for k, v in zip(met_sum, vals[1:])}


# ---- metrics for per-residue tasks (ignore_index-aware) ----------------------------------------
def token_accuracy(ignore_index: int = -100) -> Callable:
    """Accuracy over non-ignored residues; ``preds`` ``[B, K, L]`` probabilities, ``y`` ``[B, L]``."""
    def _acc(preds: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        valid = y != ignore_index
        hit = (preds.argmax(1) == y) & valid
        return hit.sum().float() / valid.sum().clamp_min(1).float()
    return _acc


def finetune(model: torch.nn.Module, train_dataloader, optimizer: torch.optim.Optimizer, epochs: int = 1,
             test_dataloader=None, loss_fn: Optional[torch.nn.Module] = None, metrics: Optional[Dict] = None,
             gradient_clipping: bool = True, gradient_clipping_thresh: float = 1.0, device=None,
             ddp=None, log: Optional[Callable[[str], None]] = None) -> Dict[str, Any]:
    """Epoch loop around :func:`train_step` / :func:`test_step` (the shape of the reference's
    commented ``train()``, ``utils.py:348-460``)."""
    loss_fn = loss_fn or torch.nn.CrossEntropyLoss(ignore_index=-100)
    metrics = metrics if metrics is not None else {"accuracy": token_accuracy()}
    results: Dict[str, Any] = {"train_loss": [], "test_loss": [], "train_metrics": [], "test_metrics": []}
    for epoch in range(epochs):
        if hasattr(getattr(train_dataloader, "sampler", None), "set_epoch"):
            train_dataloader.sampler.set_epoch(epoch)
        tl, tm = train_step(model, train_dataloader, loss_fn, optimizer, metrics, gradient_clipping,
                            gradient_clipping_thresh, device, ddp)
        results["train_loss"].append(tl)
        results["train_metrics"].append(tm)
        if test_dataloader is not None:
            vl, vm = test_step(model, test_dataloader, loss_fn, metrics, device, ddp is not None)
            results["test_loss"].append(vl)
            results["test_metrics"].append(vm)
        if log is not None and pdist.is_main():
            log(f"epoch {epoch + 1}/{epochs} train_loss={tl:.4f} {tm} "
                + (f"test_loss={results['test_loss'][-1]:.4f} {results['test_metrics'][-1]}"
                   if test_dataloader is not None else ""))
    return results


test_step.__test__ = False   # reference name; not a pytest test when imported into test modules
