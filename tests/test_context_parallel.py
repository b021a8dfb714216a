"""Context (sequence) parallelism on CPU (gloo): the L-sharded forward/backward over 3 ranks
reproduces the single-device loss, output slices and parameter gradients, in both attention
semantics (parallel/context_parallel.py; SURVEY §2.4 SP row, §5.7)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

CFG = dict(sequences_length=96, num_annotations=40, local_dim=16, global_dim=32, key_dim=8,
           num_heads=4, num_blocks=2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, semantics, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    import torch.distributed as dist
    from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
    from proteinbert_pytorch_replication_amd.models import ProteinBERT
    from proteinbert_pytorch_replication_amd.parallel.context_parallel import (
        ContextParallelProteinBERT, all_reduce_grads, cp_pretrain_loss)
    from proteinbert_pytorch_replication_amd.train.losses import pretrain_loss_torch
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    m = ProteinBERT(backend="torch", semantics=semantics, **CFG)
    X, Y, W = SyntheticUniRefGO(CFG["sequences_length"], CFG["num_annotations"], 4, "cpu", seed=7,
                                use_kernel=False).next_batch()
    # single-device oracle (identical on every rank)
    pl, pg = m(X)
    ref_loss = pretrain_loss_torch(pl, pg, Y, W, semantics=semantics)
    ref_loss.backward()
    ref_grads = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    m.zero_grad(set_to_none=True)
    for b in m.proteinBERT_blocks:
        for t in (b.global_attention_layer.Wq, b.global_attention_layer.Wk, b.global_attention_layer.Wv):
            t.grad = None
    # context-parallel
    cp = ContextParallelProteinBERT(m)
    pl_cp, pg_cp = cp(cp.shard(X["local"]), X["global"])
    loss = cp_pretrain_loss(pl_cp, pg_cp, cp.shard(Y["local"]), cp.shard(W["local"]), Y["global"], W["global"],
                            CFG["sequences_length"], world, semantics)
    loss.backward()
    tot = loss.detach().clone()
    dist.all_reduce(tot)
    params = [p for p in m.parameters()]
    all_reduce_grads(params)
    errs = {"loss": (tot - ref_loss.detach()).abs().item(),
            "probs_l": (pl_cp - cp.shard(pl.detach())).abs().max().item(),
            "probs_g": (pg_cp - pg.detach()).abs().max().item()}
    gmax = 0.0
    for n, p in m.named_parameters():
        if n in ref_grads:
            scale = max(ref_grads[n].abs().max().item(), 1e-4)   # absolute floor for ~1e-6 grads
            gmax = max(gmax, (p.grad - ref_grads[n]).abs().max().item() / scale)
    errs["grad_rel"] = gmax
    errs["heads_checked"] = any(n.endswith(".Wv") for n in ref_grads)   # registered: grad_rel covers them
    torch.save(errs, os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("semantics", ["reference", "paper"])
def test_context_parallel_matches_single_device(tmp_path, semantics):
    world = 3
    mp.start_processes(_worker, args=(world, _free_port(), semantics, str(tmp_path)), nprocs=world,
                       start_method="spawn", join=True)
    for r in range(world):
        e = torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True)
        assert e["loss"] < 1e-5, e
        assert e["probs_l"] < 1e-5, e
        assert e["probs_g"] < 1e-5, e
        assert e["grad_rel"] < 1e-4, e
        if semantics == "paper":
            assert e["heads_checked"], e


def test_halo_exchange_rejects_short_shard():
    from proteinbert_pytorch_replication_amd.parallel.context_parallel import halo_exchange
    with pytest.raises(ValueError):
        halo_exchange(torch.zeros(1, 8, 4), 20)


def _hybrid_worker(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    import torch.distributed as dist
    from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
    from proteinbert_pytorch_replication_amd.models import ProteinBERT
    from proteinbert_pytorch_replication_amd.parallel.context_parallel import (
        ContextParallelProteinBERT, all_reduce_grads, cp_pretrain_loss, make_cp_groups)
    from proteinbert_pytorch_replication_amd.train.losses import pretrain_loss_torch
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cp_size = 2
    cp_group, dp_group = make_cp_groups(cp_size)
    cfg = dict(CFG, sequences_length=64)
    torch.manual_seed(0)
    m = ProteinBERT(backend="torch", **cfg)
    batches = [SyntheticUniRefGO(64, cfg["num_annotations"], 2, "cpu", seed=20 + i, use_kernel=False).next_batch()
               for i in range(world // cp_size)]
    # oracle: DP mean of the per-batch single-device gradients
    for X, Y, W in batches:
        pl, pg = m(X)
        (pretrain_loss_torch(pl, pg, Y, W) / len(batches)).backward()
    ref = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    m.zero_grad(set_to_none=True)
    cp = ContextParallelProteinBERT(m, cp_group)
    X, Y, W = batches[rank // cp_size]
    pl, pg = cp(cp.shard(X["local"]), X["global"])
    cp_pretrain_loss(pl, pg, cp.shard(Y["local"]), cp.shard(W["local"]), Y["global"], W["global"], 64,
                     cp_size).backward()
    params = list(m.parameters())
    all_reduce_grads(params, cp_group)
    all_reduce_grads(params, dp_group, average_over=world // cp_size)
    err = max((p.grad - ref[n]).abs().max().item() / max(ref[n].abs().max().item(), 1e-4)
              for n, p in m.named_parameters() if n in ref)
    torch.save({"err": err}, os.path.join(out_dir, f"h{rank}.pt"))
    dist.destroy_process_group()


def test_cp_x_dp_groups_match_dp_mean(tmp_path):
    world = 4
    mp.start_processes(_hybrid_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       start_method="spawn", join=True)
    for r in range(world):
        e = torch.load(os.path.join(tmp_path, f"h{r}.pt"), weights_only=True)
        assert e["err"] < 1e-4, e


@pytest.mark.gpu
def test_context_parallel_gpu_rccl_long_sequence():
    """1-rank RCCL group on the GPU at L=4096 (BASELINE cfg 4 length), bf16 activations: the CP
    forward (halo path with zero padding, all-reduced LN / attention pool) equals the single-shard
    torch encoder and the backward runs."""
    import datetime
    import torch.distributed as dist
    from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
    from proteinbert_pytorch_replication_amd.models import ProteinBERT
    from proteinbert_pytorch_replication_amd.parallel.context_parallel import ContextParallelProteinBERT
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            timeout=datetime.timedelta(seconds=60), device_id=torch.device("cuda", 0))
    try:
        torch.manual_seed(0)
        m = ProteinBERT(sequences_length=4096, num_annotations=8943, local_dim=128, global_dim=512, key_dim=64,
                        num_heads=4, num_blocks=2, device="cuda", backend="torch")
        X, _, _ = SyntheticUniRefGO(4096, 8943, 2, "cuda", seed=3).next_batch()
        cp = ContextParallelProteinBERT(m, compute_dtype=torch.bfloat16)
        pl, pg = cp(cp.shard(X["local"]), X["global"])
        h, g = m.encode_torch(X["local"], X["global"], compute_dtype=torch.bfloat16)
        rl, rg = m.heads_torch(h, g)
        # bf16 activations: the two LN formulations round differently, so bound max and mean error
        assert float((pl - rl).abs().max()) < 5e-2 and float((pl - rl).abs().mean()) < 5e-3
        assert float((pg - rg).abs().max()) < 5e-2 and float((pg - rg).abs().mean()) < 5e-3
        (pl.float().square().mean() + pg.mean()).backward()
        torch.cuda.synchronize()
        assert all(torch.isfinite(p.grad).all() for p in m.parameters() if p.grad is not None)
    finally:
        dist.destroy_process_group()
