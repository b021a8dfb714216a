#!/usr/bin/env python
"""Headline benchmark: ProteinBERT pretraining throughput (sequences/s, whole job).

Metric/config from BASELINE.json: "sequences/sec (whole node) ProteinBERT
pretrain L=512 at 1/2/4/8 MI355X" on the 6-block paper config (C=128, G=512,
K=64, H=4, A=8943), random-init weights, synthetic UniRef90-shaped sequences +
GO multi-hot annotations generated and corrupted on the device every step.

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

Run as plain ``python bench.py --gpus N`` (N > 1, no WORLD_SIZE in the environment), the script
starts the N ranks itself -- ``torch.distributed.run`` as a CHILD process, launched before this
process touches the GPU -- and exits with the child's status.  Under a launcher, WORLD_SIZE must
equal ``--gpus`` or the run fails (exit 2) instead of measuring a different world.

A timed step = synthetic batch generation + corruption, forward, loss,
backward, bucketed RCCL all-reduce (N>1) and the fused Adam update.
Rank 0 prints ONE JSON line; the time is the max over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from proteinbert_pytorch_replication_amd.config import get_preset  # noqa: E402
from proteinbert_pytorch_replication_amd.models import ProteinBERT  # noqa: E402
from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO  # noqa: E402
from proteinbert_pytorch_replication_amd.parallel import dist as pdist  # noqa: E402
from proteinbert_pytorch_replication_amd.parallel.ddp import BucketedAllReduce  # noqa: E402
from proteinbert_pytorch_replication_amd.train.optim import FusedAdam  # noqa: E402
from proteinbert_pytorch_replication_amd.train.step import PretrainStep  # noqa: E402

METRIC = "sequences/sec (whole node) ProteinBERT pretrain L=512 at 1/2/4/8 MI355X"
PAPER_IMPLIED_SEQ_PER_S = 277.0  # 670M sequences / 28 days on one RTX 5000
REFERENCE_CFG1_CPU_SEQ_PER_S = 179.5  # reference cfg 1 step, 8-core CPU, survey measurement


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)   # 20-step runs spread up to 4 % on one box (r3_final2)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: preset)")
    ap.add_argument("--seq-len", type=int, default=None)
    ap.add_argument("--preset", default=None, help="config preset (default: cfg2_paper_l512; "
                    "cfg3_paper_l1024_dp8 / cfg4_long_l4096_dp8 with --seq-len 1024 / 4096; "
                    "cfg5_finetune_ss_l512_dp8 with --mode finetune)")
    ap.add_argument("--mode", default="pretrain", choices=["pretrain", "finetune"],
                    help="pretrain: the headline step; finetune: BASELINE cfg 5, frozen encoder + per-residue "
                         "8-state secondary-structure head")
    ap.add_argument("--classes", type=int, default=8, help="fine-tune head classes (secondary structure)")
    ap.add_argument("--impl", default="hip", choices=["hip", "torch", "faithful"],
                    help="hip: fused CDNA4 kernels; torch: eager bf16 oracle; faithful: reference math, eager fp32")
    ap.add_argument("--bucket-mb", type=float, default=8.0)
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="capture the whole step in a hipGraph (auto: only with PBX_GRAPH=1; eager launches "
                         "measure faster since the conv weight gradients overlap on a second stream)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--gelu", default=None, choices=["fitted", "exact"],
                    help="GELU core of the fused kernels (default: PBX_GELU or fitted): fitted = logistic fit "
                         "(max |err| 2.9e-4); exact = the erf form of the reference's nn.GELU()")
    ap.add_argument("--dp-batch-softmax", action="store_true",
                    help="reference local head: softmax over the whole DP batch (three [L, 32] all-reduces per "
                         "step; DP=N then equals the single-process batch-N*b step)")
    ap.add_argument("--semantics", default="reference", choices=["reference", "paper"],
                    help="paper: published attention/LN/softmax (per-position LayerNorm, softmax over positions)")
    return ap.parse_args()


def default_preset(mode: str, seq_len) -> str:
    """The BASELINE preset (and so the per-GPU batch) of this mode / sequence length; cfg 2 otherwise."""
    if mode == "finetune":
        return "cfg5_finetune_ss_l512_dp8"
    return {1024: "cfg3_paper_l1024_dp8", 4096: "cfg4_long_l4096_dp8"}.get(seq_len, "cfg2_paper_l512")


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(n: int) -> int:
    """Start ``n`` ranks of this script under torch.distributed.run (a child process: nothing here has
    initialised the GPU) and return its exit status."""
    import subprocess
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", os.environ.get("MASTER_PORT", str(_free_port())),
           os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd, env=env)


def main():
    a = parse()
    if a.gpus < 1:
        print("error: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(self_launch(a.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print(f"error: --gpus {a.gpus} but WORLD_SIZE={world}: refusing to measure a different world size",
              file=sys.stderr)
        sys.exit(2)
    if a.gelu is not None:
        from proteinbert_pytorch_replication_amd.ops import _lib as hiplib
        hiplib.set_gelu(a.gelu)
    info = pdist.init_distributed()
    dev = info.device
    cfg = get_preset(a.preset or default_preset(a.mode, a.seq_len))
    mcfg = cfg.model
    L = a.seq_len or mcfg.sequences_length
    B = a.batch or cfg.train.batch_size
    torch.manual_seed(a.seed)
    if a.impl == "hip" and dev.type != "cuda":
        a.impl = "torch"            # CPU rehearsal (gloo ranks): the fused kernels need a GPU
    backend = "hip" if a.impl == "hip" else "torch"
    model = ProteinBERT(sequences_length=L, num_annotations=mcfg.num_annotations, local_dim=mcfg.local_dim,
                        global_dim=mcfg.global_dim, key_dim=mcfg.key_dim, num_heads=mcfg.num_heads,
                        num_blocks=mcfg.num_blocks, device=dev,
                        backend=backend, semantics=a.semantics)
    if a.mode == "finetune":
        return finetune_bench(a, info, model, L, B, mcfg)
    opt = FusedAdam(model.parameters(), lr=2e-4)
    ddp = BucketedAllReduce(opt.arena, bucket_mb=a.bucket_mb) if info.distributed else None
    if ddp is not None:
        ddp.broadcast_parameters(model)
    if a.dp_batch_softmax and info.distributed:
        from proteinbert_pytorch_replication_amd.parallel import batch_softmax
        batch_softmax.enable()
    # bf16 activations on the GPU; the CPU rehearsal path (gloo ranks, BASELINE cfg 1) computes in fp32
    dtype = torch.float32 if (a.impl == "faithful" or dev.type != "cuda") else torch.bfloat16
    step = PretrainStep(model, opt, ddp, compute_dtype=dtype)
    if a.impl == "faithful":
        # reference computation as written: literal Q/K/softmax attention, fp32, eager
        def faithful_loss(X, Y, W, return_parts=False):
            from proteinbert_pytorch_replication_amd.train.losses import pretrain_loss_torch
            h, g = model.encode_torch(X["local"], X["global"], torch.float32, faithful_attention=True)
            pl, pg = model.heads_torch(h, g)
            return pretrain_loss_torch(pl, pg, Y, W, return_parts=return_parts)
        step.loss = faithful_loss
    gen = SyntheticUniRefGO(L, mcfg.num_annotations, B, dev, seed=a.seed + 1000 * info.rank)
    batches = gen.next_batch
    if dev.type == "cuda" and os.environ.get("PBX_PREFETCH", "0") == "1":
        # PBX_PREFETCH=1: the next step's synthetic batch is generated on a side stream beside this step
        # (train.step.PrefetchedBatches); measured neutral (-0.1 %, 3 same-box rounds), so the default
        # generates it at the head of each step
        from proteinbert_pytorch_replication_amd.train.step import PrefetchedBatches
        batches = PrefetchedBatches(gen.next_batch, dev)

    def one():
        X, Y, W = batches()
        return step(X, Y, W)

    use_graph = a.graph == "on" or (a.graph == "auto" and dev.type == "cuda" and a.impl == "hip" and
                                     os.environ.get("PBX_GRAPH") == "1")
    graphed = False
    if use_graph:
        from proteinbert_pytorch_replication_amd.train.step import GraphedStep
        try:
            one = GraphedStep(step, gen.next_batch, warmup=2)
            graphed = True
        except Exception as e:  # capture unsupported here: run eagerly
            print(f"warning: hipGraph capture failed ({type(e).__name__}: {e}); running eagerly", file=sys.stderr)

    dt, loss = _timed(one, a, info, dev)
    final_loss = float(loss.item())
    n = info.world_size
    value = n * B * a.steps / dt
    if info.is_main:
        out = {"metric": METRIC, "value": round(value, 2), "unit": "sequences/s", "n_gpus": n,
               "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(1000 * dt / a.steps, 3),
               "higher_is_better": True, "scaling": "weak",
               "vs_baseline": round(value / PAPER_IMPLIED_SEQ_PER_S, 2),
               "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
               "data": _data_label(dev),
               "config": {"model": f"ProteinBERT paper config: {mcfg.num_blocks} blocks, d_local={mcfg.local_dim}, "
                                   f"d_global={mcfg.global_dim}, key_dim={mcfg.key_dim}, heads={mcfg.num_heads}, "
                                   f"annotations={mcfg.num_annotations}, semantics={a.semantics}",
                          "global_batch": B * n, "per_gpu_batch": B, "seq_len": L, "parallelism": f"dp{n}",
                          "impl": a.impl, "hip_graph": graphed},
               "world_size": n, "backend": info.backend if n > 1 else "single",
               "rccl_env": getattr(info, "rccl_env", None),
               "dp_transport": ddp.transport if ddp is not None else "none",
               "dp_batch_softmax": bool(a.dp_batch_softmax and n > 1),
               "gelu": _gelu_label(a.impl),
               "device": _device_label(dev), "final_loss": round(final_loss, 5),
               # the reference reduces its loss in float64 (float64 weights, utils.py:293-294); the fused
               # heads reduce in fp32: < 1e-6 relative at this shape (tests/test_loss_precision.py)
               "loss_reduction": "fp32 (reference: float64)" if a.impl == "hip" else "as the weights' dtype"}
        if dev.type == "cuda":
            out["peak_mem_gib"] = round(torch.cuda.max_memory_allocated(dev) / 2**30, 2)
        if dev.type != "cuda" and a.preset == "cfg1_cpu_smoke":
            # BASELINE cfg 1 is a CPU config: compare with the reference step measured on a CPU
            out["vs_baseline"] = round(value / REFERENCE_CFG1_CPU_SEQ_PER_S, 2)
            out["baseline"] = "reference modules.py cfg 1 step on an 8-core CPU (BASELINE.md)"
        print(json.dumps(out), flush=True)
    if ddp is not None:
        ddp.close()
    pdist.destroy()


def _gelu_label(impl: str) -> str:
    if impl != "hip":
        return "exact (torch nn.GELU)"
    from proteinbert_pytorch_replication_amd.ops import _lib as hiplib
    return {"fitted": "fitted logistic core in the fused kernels (max |err| 2.9e-4 vs erf; --gelu exact for erf)",
            "exact": "exact erf form (A&S 7.1.26, |err| <= 1.5e-7)"}.get(hiplib.gelu_mode(), hiplib.HIP_LIB)


def _device_label(dev) -> str:
    if dev.type != "cuda":
        return f"cpu ({torch.get_num_threads()} threads)"
    return torch.cuda.get_device_name(dev)


def _data_label(dev) -> str:
    where = "generated on the device by HIP kernels" if dev.type == "cuda" else "generated on the host CPU"
    return (f"synthetic: UniRef90-shaped sequences + 8943-dim GO multi-hot, {where} and corrupted every step; "
            "random-init weights")


def _timed(one, a, info, dev):
    for _ in range(a.warmup):
        loss = one()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    pdist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = one()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    pdist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    return pdist.all_reduce_max(time.perf_counter() - t0, dev), loss


def finetune_bench(a, info, encoder, L, B, mcfg):
    """BASELINE cfg 5: the fine-tune step of a frozen pretrained encoder (random-init here) with a
    per-residue secondary-structure head (reference train_step contract, utils.py:110-168: CE over
    dim 1, gradient clipping at 1.0), synthetic tokens/labels; DP all-reduces the head gradients."""
    import torch.nn.functional as F
    from proteinbert_pytorch_replication_amd.models.finetune import ProteinBERTForTokenClassification
    dev = info.device
    model = ProteinBERTForTokenClassification(encoder, n_classes=a.classes, freeze_encoder=True)
    opt = FusedAdam([p for p in model.parameters() if p.requires_grad], lr=1e-3)
    ddp = BucketedAllReduce(opt.arena, bucket_mb=a.bucket_mb) if info.distributed else None
    if ddp is not None:
        ddp.broadcast_parameters(model)
    gen = SyntheticUniRefGO(L, mcfg.num_annotations, B, dev, seed=a.seed + 1000 * info.rank)
    g = torch.Generator(device=dev)
    g.manual_seed(a.seed + 7 + info.rank)

    def one():
        X, Y, _ = gen.next_batch()
        y = torch.randint(0, a.classes, Y["local"].shape, device=dev, generator=g)
        y = torch.where(Y["local"] == 0, torch.full_like(y, -100), y)          # padding is ignored
        opt.zero_grad()
        loss = F.cross_entropy(model(X), y, ignore_index=-100)
        loss.backward()
        if ddp is not None:
            ddp.finish(average=False)
        opt.clip_grad_norm_(1.0)
        opt.step()
        return loss.detach()

    dt, loss = _timed(one, a, info, dev)
    n = info.world_size
    value = n * B * a.steps / dt
    if info.is_main:
        out = {"metric": "sequences/sec (whole node) ProteinBERT fine-tune (frozen encoder + per-residue "
                         f"{a.classes}-state head) L={L}", "value": round(value, 2), "unit": "sequences/s",
               "n_gpus": n, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(1000 * dt / a.steps, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
               "dtype": "bf16" if dev.type == "cuda" else "fp32",
               "data": _data_label(dev).replace("GO multi-hot", "GO multi-hot, random per-residue labels"),
               "world_size": n,
               "config": {"model": f"ProteinBERT paper config encoder (frozen) + Linear({mcfg.local_dim}+"
                                   f"{mcfg.global_dim} -> {a.classes}) per residue",
                          "global_batch": B * n, "per_gpu_batch": B, "seq_len": L, "parallelism": f"dp{n}",
                          "impl": a.impl}, "final_loss": round(float(loss.item()), 5)}
        print(json.dumps(out), flush=True)
    if ddp is not None:
        ddp.close()
    pdist.destroy()


if __name__ == "__main__":
    main()
