"""``pretrain()``: the reference's training loop API on the MI355X engine.

Same signature and defaults as the reference (``ProteinBERT/utils.py:220-345``):
``pretrain(model, train_dataloader, optimizer, local_loss_fn, global_loss_fn,
max_batch_iterations, save_path, nb_iterations_checkpoint=1000,
optim_scheduler_patience=25, warmup_duration=10000, loaded_checkpoint=None,
device=...) -> {"train_loss": [...]}``, same log line, same checkpoint
files and keys.  Differences (all additive):

* a working warmup -> plateau schedule (reference SequentialLR is broken on
  torch 2.10);
* data parallel over RCCL when launched with torchrun (rank-0 logging and
  checkpoints, bucketed overlapped all-reduce);
* the loss is read back to the host only every ``log_every`` steps (the
  reference syncs every step);
* resume restores RNG state and attention heads (``extra_state``);
* fault injection (``PBX_FAULT_AT_STEP``) and automatic resume from the latest
  checkpoint (``resume="latest"``) for elastic restarts.
"""
from __future__ import annotations

import logging
import os
import time
from typing import Any, Dict, Optional

import torch

from ..utils.profiling import StepProfiler, marker
from ..parallel import dist as pdist
from ..parallel.ddp import BucketedAllReduce
from .checkpoint import (CheckpointWriter, build_checkpoint, checkpoint_name, latest_checkpoint, load_checkpoint,
                         rng_state, save_final_model, set_rng_state)
from .optim import FusedAdam
from .schedulers import WarmupThenPlateau
from .step import PretrainStep
from ..utils.metrics import MetricsWriter

log = logging.getLogger("pbx.pretrain")


def _to_device(d: Dict[str, torch.Tensor], device) -> Dict[str, torch.Tensor]:
    return {k: v.to(device, non_blocking=True) for k, v in d.items()}


def _loader_state(loader) -> Dict[str, Any]:
    """Resumable loaders (NativeStoreLoader) store their cursor in the checkpoint."""
    sd = getattr(loader, "state_dict", None)
    return {"loader": sd()} if callable(sd) and not isinstance(loader, torch.nn.Module) else {}


def _maybe_fuse_optimizer(model, optimizer) -> torch.optim.Optimizer:
    if isinstance(optimizer, FusedAdam) or type(optimizer) is not torch.optim.Adam:
        return optimizer
    g = optimizer.param_groups
    if len(g) != 1 or g[0].get("amsgrad") or g[0].get("maximize"):
        return optimizer
    fused = FusedAdam(g[0]["params"], lr=g[0]["lr"], betas=g[0]["betas"], eps=g[0]["eps"],
                      weight_decay=g[0]["weight_decay"])
    if optimizer.state:
        fused.load_state_dict(optimizer.state_dict())
    return fused


def pretrain(model: torch.nn.Module, train_dataloader, optimizer: torch.optim.Optimizer,
             local_loss_fn: Optional[torch.nn.Module] = None, global_loss_fn: Optional[torch.nn.Module] = None,
             max_batch_iterations: int = 250, save_path: str = ".", nb_iterations_checkpoint: int = 1000,
             optim_scheduler_patience: int = 25, warmup_duration: int = 10000,
             loaded_checkpoint: Optional[Dict[str, Any]] = None, device=None, *,
             log_every: int = 1, bucket_mb: float = 8.0, compute_dtype="auto", grad_clip: Optional[float] = None,
             async_checkpoint: bool = False, metrics_path: Optional[str] = None, resume: str = "none",
             fuse_optimizer: bool = True, final_save: bool = True, profile_steps: Optional[str] = None,
             profile_dir: Optional[str] = None, zero_optimizer: bool = False,
             comm_dtype="fp32", tensorboard_dir: Optional[str] = None,
             dp_batch_softmax: bool = False) -> Dict[str, Any]:
    info = pdist.init_distributed()
    if device is None:
        device = info.device
    device = torch.device(device)
    model.to(device)
    if fuse_optimizer:
        optimizer = _maybe_fuse_optimizer(model, optimizer)
    results: Dict[str, Any] = {"train_loss": [], "optimizer": optimizer}

    ddp = None
    if info.distributed:
        from ..parallel.zero import ZeroFusedAdam
        if not isinstance(optimizer, FusedAdam):
            raise ValueError("data-parallel pretrain needs FusedAdam (flat gradient arena)")
        if zero_optimizer and not isinstance(optimizer, ZeroFusedAdam):
            # ZeRO-1: Adam moments sharded over the DP ranks (parallel/zero.py); reduce-scatter at step()
            g = optimizer.param_groups[0]
            zopt = ZeroFusedAdam(optimizer.arena, lr=g["lr"], betas=g["betas"], eps=g["eps"],
                                 weight_decay=g["weight_decay"])
            if optimizer.step_count:
                zopt.load_state_dict(optimizer.state_dict())
            optimizer = zopt
            results["optimizer"] = optimizer
        if isinstance(optimizer, ZeroFusedAdam):
            pdist.broadcast_module(model)
        else:
            cdt = comm_dtype if isinstance(comm_dtype, torch.dtype) else \
                {"fp32": torch.float32, "bf16": torch.bfloat16}[comm_dtype]
            ddp = BucketedAllReduce(optimizer.arena, bucket_mb=bucket_mb, comm_dtype=cdt)
            ddp.broadcast_parameters(model)
        if dp_batch_softmax:
            # the reference local head normalises over the batch axis: share it over the DP ranks so DP=N
            # with micro-batch b is the batch-N*b step (modules.py:277-284)
            from ..parallel import batch_softmax
            batch_softmax.enable()

    scheduler = WarmupThenPlateau(optimizer, warmup_duration=warmup_duration, patience=optim_scheduler_patience)
    step_fn = PretrainStep(model, optimizer, ddp, local_loss_fn, global_loss_fn, compute_dtype, grad_clip)
    writer = CheckpointWriter(save_path, async_checkpoint, is_main=info.is_main)
    metrics = MetricsWriter(metrics_path if info.is_main else None)
    tb = None
    if tensorboard_dir and info.is_main:
        from ..utils.tensorboard import SummaryWriter
        tb = SummaryWriter(tensorboard_dir)

    if loaded_checkpoint is None and resume == "latest":
        path = latest_checkpoint(save_path)
        if path is not None:
            log.info("Resuming from %s", path)
            loaded_checkpoint = load_checkpoint(path)
    current = 0
    if loaded_checkpoint is not None:
        logging.info("Loading checkpoint...")
        current = int(loaded_checkpoint["current_batch_iteration"])
        model.load_state_dict(loaded_checkpoint["model_state_dict"])
        optimizer.load_state_dict(loaded_checkpoint["optimizer_state_dict"])
        scheduler.load_state_dicts(loaded_checkpoint)
        extra = loaded_checkpoint.get("extra_state", {})
        if "attention_heads" in extra:
            model.load_attention_heads_state(extra["attention_heads"])
        if "rng" in extra and extra.get("world_size", 1) == info.world_size:
            set_rng_state(extra["rng"], device)
        if "loader" in extra and hasattr(train_dataloader, "load_state_dict") \
                and extra.get("world_size", 1) == info.world_size:
            train_dataloader.load_state_dict(extra["loader"])
        logging.info("Checkpoint loaded!")

    profiler = StepProfiler.from_spec(profile_steps, profile_dir or save_path, info.rank)
    fault_at = int(os.environ.get("PBX_FAULT_AT_STEP", "0") or 0)
    fault_rank = int(os.environ.get("PBX_FAULT_RANK", "0") or 0)
    model.train()
    loss_acc = torch.zeros((), dtype=torch.float32, device=device)
    parts_acc = torch.zeros(2, dtype=torch.float32, device=device)      # local (CE), global (BCE)
    from ..utils.flops import mfu, train_flops_per_sequence
    cfg = getattr(model, "config", None)
    n_acc = 0
    t_last = time.time()
    last_loss = float("nan")
    while current < max_batch_iterations:
        progressed = False
        for X, Y, W in train_dataloader:
            progressed = True
            start_time = time.time()
            X, Y, W = _to_device(X, device), _to_device(Y, device), _to_device(W, device)
            if profiler is not None:
                profiler.before_step(current + 1)
            with marker("pbx/step"):
                loss = step_fn(X, Y, W)
            loss_acc += loss.float()
            if step_fn.last_parts is not None:
                parts_acc[0] += step_fn.last_parts[0].float()
                parts_acc[1] += step_fn.last_parts[1].float()
            n_acc += 1
            current += 1
            if profiler is not None:
                profiler.after_step(current)
                if profiler.trace_path:
                    results["profile_trace"] = profiler.trace_path
            if scheduler.in_warmup:
                scheduler.step(None)
            if fault_at and current == fault_at and info.rank == fault_rank:
                log.error("PBX_FAULT_AT_STEP=%d: injected failure on rank %d", fault_at, info.rank)
                os._exit(17)
            if current % log_every == 0 or current >= max_batch_iterations:
                if info.distributed:
                    pdist.all_reduce_mean_(loss_acc)
                    pdist.all_reduce_mean_(parts_acc)
                last_loss = float(loss_acc.item()) / max(1, n_acc)
                part_l, part_g = (float(v) / max(1, n_acc) for v in parts_acc.tolist())
                now = time.time()
                dt = (now - t_last) / max(1, n_acc)
                t_last = now
                for _ in range(n_acc):
                    results["train_loss"].append(last_loss)
                if info.is_main:
                    logging.info(f"Current batch iteration: {current} | Train loss: {last_loss:.4f} | "
                                 f"Learning rate: {scheduler.get_last_lr()[0]} | "
                                 f"Batch Iteration time: {dt:.4f} seconds")
                    seq_s = X["local"].shape[0] * info.world_size / max(dt, 1e-9)
                    Ls = X["local"].shape[1]
                    rec = dict(step=current, loss=last_loss, loss_local=part_l, loss_global=part_g,
                               lr=scheduler.get_last_lr()[0], step_time_s=dt, seq_per_s=seq_s,
                               tokens_per_s=seq_s * Ls)
                    if cfg is not None:
                        rec["mfu"] = mfu(train_flops_per_sequence(cfg, Ls), seq_s, n_devices=info.world_size)
                    if device.type == "cuda":
                        rec["max_mem_gb"] = torch.cuda.max_memory_allocated(device) / 2 ** 30
                    metrics.write(**rec)
                    if tb is not None:
                        tb.add_scalars({"train/loss": last_loss, "train/lr": scheduler.get_last_lr()[0],
                                        "perf/step_time_s": dt, "perf/seq_per_s": seq_s}, current)
                if not scheduler.in_warmup:
                    # plateau patience counts log intervals (== steps at log_every=1, the reference)
                    scheduler.step(last_loss)
                loss_acc.zero_()
                parts_acc.zero_()
                n_acc = 0
            if current >= max_batch_iterations:
                break
            if current % nb_iterations_checkpoint == 0:
                ckpt = build_checkpoint(current, model, optimizer, scheduler, last_loss,
                                        extra={"rng": rng_state(device), "world_size": info.world_size,
                                               "data_cursor": current, **_loader_state(train_dataloader)})
                writer.save(ckpt, checkpoint_name(current))
                pdist.barrier()
        if not progressed:
            raise RuntimeError("train_dataloader yielded no batches")
    writer.wait()
    metrics.close()
    if tb is not None:
        tb.close()
    if final_save:
        results["final_model_path"] = save_final_model(model, save_path, info.is_main)
    return results
