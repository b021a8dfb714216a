"""Data parallelism on CPU (gloo, world_size 2): bucketed all-reduce step == averaged-gradient step,
rank-0-only checkpointing under DP pretrain, and fault injection + resume."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
from proteinbert_pytorch_replication_amd.models import ProteinBERT
from proteinbert_pytorch_replication_amd.train.optim import FusedAdam
from proteinbert_pytorch_replication_amd.train.step import PretrainStep

CFG = dict(sequences_length=32, num_annotations=40, local_dim=16, global_dim=32, key_dim=8,
           num_heads=4, num_blocks=2)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank, world, port):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))


def _dp_worker(rank, world, port, out_dir, steps, comm="fp32", overlap=True):
    _env(rank, world, port)
    os.environ["PBX_DP_OVERLAP_OPT"] = "1" if overlap else "0"
    torch.set_num_threads(1)
    from proteinbert_pytorch_replication_amd.parallel import dist as pdist
    from proteinbert_pytorch_replication_amd.parallel.ddp import BucketedAllReduce
    info = pdist.init_distributed(device="cpu")
    torch.manual_seed(0)
    m = ProteinBERT(backend="torch", **CFG)
    opt = FusedAdam(m.parameters(), lr=1e-2)
    ddp = BucketedAllReduce(opt.arena, bucket_mb=0.004,     # many small buckets
                            comm_dtype=torch.bfloat16 if comm == "bf16" else torch.float32)
    assert len(ddp.buckets) > 3
    ddp.broadcast_parameters(m)
    step = PretrainStep(m, opt, ddp)
    gen = SyntheticUniRefGO(CFG["sequences_length"], CFG["num_annotations"], 4, "cpu", seed=100 + rank,
                            use_kernel=False)
    for _ in range(steps):
        step(*gen.next_batch())
    assert step.overlapped_optimizer() == overlap
    torch.save({k: v.detach().clone() for k, v in m.state_dict().items()},
               os.path.join(out_dir, f"rank{rank}.pt"))
    pdist.destroy()


@pytest.mark.parametrize("comm", ["fp32", "bf16"])
def test_dp_bucketed_allreduce_equals_averaged_gradients(tmp_path, comm):
    """comm=bf16: every bucket reduced through a bf16 copy (DistConfig.comm_dtype)."""
    steps, world = 3, 2
    mp.start_processes(_dp_worker, args=(world, _free_port(), str(tmp_path), steps, comm), nprocs=world,
                       start_method="spawn", join=True)
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    for k in r0:
        assert torch.equal(r0[k], r1[k]), k           # replicas stay bit-identical
    # single-process oracle: mean of the per-rank gradients, same Adam
    torch.manual_seed(0)
    m = ProteinBERT(backend="torch", **CFG)
    opt = FusedAdam(m.parameters(), lr=1e-2)
    step = PretrainStep(m, opt)
    gens = [SyntheticUniRefGO(CFG["sequences_length"], CFG["num_annotations"], 4, "cpu", seed=100 + r,
                              use_kernel=False) for r in range(world)]
    opt.grad_scale = 1.0 / world
    for _ in range(steps):
        opt.zero_grad()
        for g in gens:
            step.loss(*g.next_batch()).backward()
        opt.step()
    for k, v in m.state_dict().items():
        if k == "pretraining_local_output.0.bias":
            # its true gradient is exactly 0 (softmax over the batch axis): Adam turns
            # summation-order noise into lr-sized steps, so only the update bound is meaningful
            assert float((r0[k] - v).abs().max()) <= 2 * 1e-2 * steps
            continue
        if comm == "bf16":
            # bf16-rounded gradient sums: Adam's normalised steps stay within lr of the fp32 oracle
            d = (r0[k] - v).abs()
            assert float(d.max()) <= 2 * 1e-2 * steps, k
            assert float((d > 1e-3).float().mean()) < 0.05, k
            continue
        torch.testing.assert_close(r0[k], v, rtol=1e-4, atol=2e-5, msg=k)


def test_dp_overlapped_optimizer_bitwise_equals_whole_arena_step(tmp_path):
    """Per-bucket Adam beside the last bucket's all-reduce (BucketedAllReduce.finish_and_step) gives
    bitwise the parameters of finish() + one whole-arena update (Adam is element-wise)."""
    steps, world = 3, 2
    for tag, ov in (("ov", True), ("whole", False)):
        d = tmp_path / tag
        d.mkdir()
        mp.start_processes(_dp_worker, args=(world, _free_port(), str(d), steps, "fp32", ov), nprocs=world,
                           start_method="spawn", join=True)
    a = torch.load(tmp_path / "ov" / "rank0.pt", weights_only=True)
    b = torch.load(tmp_path / "whole" / "rank0.pt", weights_only=True)
    for k in a:
        assert torch.equal(a[k], b[k]), k


def _nonfinite_worker(rank, world, port, out_dir):
    """Rank 1 poisons one gradient of the FIRST bucket: every rank must skip every bucket's update."""
    _env(rank, world, port)
    torch.set_num_threads(1)
    from proteinbert_pytorch_replication_amd.parallel import dist as pdist
    from proteinbert_pytorch_replication_amd.parallel.ddp import BucketedAllReduce
    pdist.init_distributed(device="cpu")
    torch.manual_seed(0)
    m = ProteinBERT(backend="torch", **CFG)
    opt = FusedAdam(m.parameters(), lr=1e-2)
    ddp = BucketedAllReduce(opt.arena, bucket_mb=0.004)
    step = PretrainStep(m, opt, ddp)
    before = opt.arena.data.clone()
    first = opt.arena.params[0]
    if rank == 1:
        first.register_hook(lambda g: g * float("nan"))
    step(*SyntheticUniRefGO(CFG["sequences_length"], CFG["num_annotations"], 4, "cpu", seed=100 + rank,
                            use_kernel=False).next_batch())
    assert torch.equal(opt.arena.data, before), f"rank {rank} updated despite a non-finite gradient"
    pdist.destroy()


def test_dp_overlapped_optimizer_skips_all_buckets_on_nonfinite(tmp_path):
    mp.start_processes(_nonfinite_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, start_method="spawn",
                       join=True)


def _overflow_worker(rank, world, port, out_dir, where):
    """Both ranks hold a FINITE gradient of 3e38 in one element; their SUM overflows fp32.  The local test
    (|g| >= FLT_MAX / world) flags it before any all-reduce, so wherever the element sits (first or last
    bucket) the whole step is skipped on every rank: no Inf reaches the parameters and no step is applied
    to only part of the arena."""
    _env(rank, world, port)
    torch.set_num_threads(1)
    from proteinbert_pytorch_replication_amd.parallel import dist as pdist
    from proteinbert_pytorch_replication_amd.parallel.ddp import BucketedAllReduce
    pdist.init_distributed(device="cpu")
    torch.manual_seed(0)
    m = ProteinBERT(backend="torch", **CFG)
    opt = FusedAdam(m.parameters(), lr=1e-2)
    ddp = BucketedAllReduce(opt.arena, bucket_mb=0.004)
    step = PretrainStep(m, opt, ddp)
    before = opt.arena.data.clone()
    p = opt.arena.params[0] if where == "head" else opt.arena.params[-1]

    def big(g):
        g = g.clone()
        g.view(-1)[0] = 3e38
        return g
    p.register_hook(big)
    step(*SyntheticUniRefGO(CFG["sequences_length"], CFG["num_annotations"], 4, "cpu", seed=100 + rank,
                            use_kernel=False).next_batch())
    assert torch.isfinite(opt.arena.data).all(), f"rank {rank}: an overflowed sum reached the parameters"
    assert torch.equal(opt.arena.data, before), f"rank {rank} updated part of the arena despite an overflowing sum"
    torch.save(opt.arena.data, os.path.join(out_dir, f"rank{rank}.pt"))
    pdist.destroy()


@pytest.mark.parametrize("where", ["head", "tail"])
def test_dp_overlapped_optimizer_catches_summed_overflow(tmp_path, where):
    mp.start_processes(_overflow_worker, args=(2, _free_port(), str(tmp_path), where), nprocs=2,
                       start_method="spawn", join=True)
    a = torch.load(tmp_path / "rank0.pt", weights_only=True)
    b = torch.load(tmp_path / "rank1.pt", weights_only=True)
    assert torch.equal(a, b)                         # every rank took the same decision


def _pretrain_worker(rank, world, port, save, zero=False):
    _env(rank, world, port)
    torch.set_num_threads(1)
    from proteinbert_pytorch_replication_amd.train.pretrain import pretrain
    torch.manual_seed(0)
    m = ProteinBERT(backend="torch", **CFG)
    gen = SyntheticUniRefGO(CFG["sequences_length"], CFG["num_annotations"], 4, "cpu", seed=rank, use_kernel=False)
    pretrain(m, gen, torch.optim.Adam(m.parameters(), lr=1e-3), max_batch_iterations=5, save_path=save,
             nb_iterations_checkpoint=2, warmup_duration=2, device="cpu", zero_optimizer=zero)


@pytest.mark.parametrize("zero", [False, True])
def test_dp_pretrain_rank0_checkpoints(tmp_path, zero):
    mp.start_processes(_pretrain_worker, args=(2, _free_port(), str(tmp_path), zero), nprocs=2,
                       start_method="spawn", join=True)
    files = sorted(os.listdir(tmp_path))
    assert "proteinbert_pretraining_checkpoint_2.pt" in files and "proteinbert_pretraining_checkpoint_4.pt" in files
    assert len([f for f in files if f.startswith("proteinbert_pretrained_model_")]) == 1
    blob = torch.load(tmp_path / "proteinbert_pretraining_checkpoint_4.pt", weights_only=False)
    assert blob["extra_state"]["world_size"] == 2
    # ZeRO-1 checkpoints hold the gathered (full-size) moments, same format as the all-reduce path
    m = ProteinBERT(backend="torch", **CFG)
    shapes = [p.shape for p in m.parameters()]
    st = blob["optimizer_state_dict"]["state"]
    assert len(st) == len(shapes)
    assert sorted(tuple(v["exp_avg"].shape) for v in st.values()) == sorted(tuple(s) for s in shapes)


SCRIPT = r'''
import sys, torch
sys.path.insert(0, {root!r})
from proteinbert_pytorch_replication_amd.models import ProteinBERT
from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
from proteinbert_pytorch_replication_amd.train.pretrain import pretrain
torch.manual_seed(0)
m = ProteinBERT(backend="torch", **{cfg!r})
gen = SyntheticUniRefGO(32, 40, 4, "cpu", seed=1, use_kernel=False)
r = pretrain(m, gen, torch.optim.Adam(m.parameters(), lr=1e-3), max_batch_iterations=6, save_path={save!r},
             nb_iterations_checkpoint=2, warmup_duration=2, device="cpu", resume="latest", final_save=False)
print("STEPS", len(r["train_loss"]))
'''


def test_fault_injection_then_resume_from_latest(tmp_path):
    code = SCRIPT.format(root=ROOT, cfg=CFG, save=str(tmp_path))
    env = dict(os.environ, PBX_FAULT_AT_STEP="5", PBX_FAULT_RANK="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 17, r.stderr[-2000:]
    assert (tmp_path / "proteinbert_pretraining_checkpoint_4.pt").exists()
    env.pop("PBX_FAULT_AT_STEP")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "STEPS 2" in r.stdout          # resumed at iteration 4, ran 5 and 6


def test_bucketer_counts_each_parameter_once():
    """A fused backward announces the gradients it wrote in place (notify_grads_ready) and autograd
    then still runs those parameters' post-accumulate hooks: each parameter must count once toward
    its bucket, else buckets are reduced before their last gradient is written (found on 2 GPU
    ranks: the global->local weights were reduced before their in-place write)."""
    import datetime
    import torch.distributed as dist
    from proteinbert_pytorch_replication_amd.parallel.ddp import BucketedAllReduce
    from proteinbert_pytorch_replication_amd.train.arena import FlatArena
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            timeout=datetime.timedelta(seconds=30))
    try:
        params = [torch.nn.Parameter(torch.randn(300)) for _ in range(6)]
        arena = FlatArena(params)
        ddp = BucketedAllReduce(arena, bucket_mb=600 * 4 / 2 ** 20, force=True)
        assert len(ddp.buckets) >= 2
        launched = []
        ddp._launch = lambda b: launched.append(b)
        first = [p for p in arena.params if ddp.param_bucket[arena.param_index()[id(p)]] == 0]
        # direct announcement of ONE parameter of bucket 0, then its autograd hook as well
        ddp._on_direct_grads(first[:1])
        ddp._make_hook(arena.param_index()[id(first[0])])(first[0])
        assert launched == [] and min(ddp._pending) >= 0
        for p in first[1:]:
            ddp._make_hook(arena.param_index()[id(p)])(p)
        assert launched == [0]
        ddp.start_step()
        assert ddp._pending == ddp.bucket_nparams and not any(ddp._ready)
    finally:
        dist.destroy_process_group()


def test_rccl_node_defaults_respect_environment(monkeypatch):
    """single-node RCCL defaults are applied only where the environment is silent, never on
    multi-node jobs, and not at all with PBX_RCCL_DEFAULTS=0."""
    from proteinbert_pytorch_replication_amd.parallel import dist as pdist
    for k in pdist.RCCL_NODE_DEFAULTS:
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("NCCL_MIN_NCHANNELS", "32")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    applied = pdist.rccl_node_defaults(8)
    assert os.environ["NCCL_MIN_NCHANNELS"] == "32" and "NCCL_MIN_NCHANNELS" not in applied
    assert os.environ["HSA_NO_SCRATCH_RECLAIM"] == "1"
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    assert pdist.rccl_node_defaults(8) is None                 # two nodes
    monkeypatch.setenv("PBX_RCCL_DEFAULTS", "0")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert pdist.rccl_node_defaults(8) is None


def _uid_worker(rank, world, port, out_dir):
    """The direct RCCL communicator's unique-id hand-off (parallel/rccl.py) through the process group's store:
    rank 0's id reaches every rank byte for byte (no GPU needed for this part)."""
    _env(rank, world, port)
    from proteinbert_pytorch_replication_amd.parallel import dist as pdist
    from proteinbert_pytorch_replication_amd.parallel import rccl
    pdist.init_distributed(device="cpu")
    blob = bytes(range(128)) + b""
    got = rccl.exchange_unique_id(rank, "pbx_test_uid/0", lambda: blob)
    got2 = rccl.exchange_unique_id(rank, "pbx_test_uid/1", lambda: bytes(reversed(blob)))
    assert rccl.wanted() is False              # gloo: the buckets stay on torch.distributed
    with open(os.path.join(out_dir, f"uid{rank}.bin"), "wb") as f:
        f.write(got + got2)
    pdist.destroy()


def test_rccl_unique_id_exchange(tmp_path):
    mp.start_processes(_uid_worker, args=(3, _free_port(), str(tmp_path)), nprocs=3, start_method="spawn", join=True)
    blobs = [open(tmp_path / f"uid{r}.bin", "rb").read() for r in range(3)]
    assert blobs[0] == blobs[1] == blobs[2] == bytes(range(128)) + bytes(reversed(range(128)))
