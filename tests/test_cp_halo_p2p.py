"""The fused-executor CP halo exchange (parallel/cp_fused.py ``halo_rows_many``) on CPU gloo: neighbour
isend / irecv only, checked against the zero-padded window of the full tensor, on the world group (3
ranks) and on a sub-group whose group ranks differ from the global ranks (ranks 1..3 of 4)."""
import os
import socket

import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, sub, out_dir):
    import torch.distributed as dist
    from proteinbert_pytorch_replication_amd.parallel.cp_fused import CPShard
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    group = None
    members = list(range(world))
    if sub:
        members = list(range(1, world))
        group = dist.new_group(members)
    ok = True
    if rank in members:
        B, L, C, H = 2, 96, 8, 20
        full = [torch.randn(B, L, C, generator=torch.Generator().manual_seed(k)) for k in range(3)]
        cp = CPShard(L, group=group, halo=H)
        got = cp.halo_rows_many(*[cp.shard(x) for x in full])
        single = cp.halo_rows(cp.shard(full[0]))
        for x, g in zip(full, got):
            pad = torch.cat([torch.zeros(B, H, C), x, torch.zeros(B, H, C)], dim=1)
            want = pad[:, cp.start:cp.start + cp.shard_len + 2 * H]
            ok = ok and g.shape == want.shape and torch.equal(g, want)
        ok = ok and torch.equal(single, got[0])
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write("ok" if ok else "bad")
    dist.barrier()
    dist.destroy_process_group()


def _run(tmp_path, world, sub):
    mp.start_processes(_worker, args=(world, _free_port(), sub, str(tmp_path)), nprocs=world,
                       start_method="spawn", join=True)
    for r in range(world):
        assert (tmp_path / f"r{r}.txt").read_text() == "ok", r


def test_halo_p2p_world_group(tmp_path):
    _run(tmp_path, 3, False)


def test_halo_p2p_subgroup(tmp_path):
    _run(tmp_path, 4, True)


def _softmax_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    from proteinbert_pytorch_replication_amd.ops.paper_track import _cp_softmax_combine
    from proteinbert_pytorch_replication_amd.parallel.cp_fused import CPShard
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    B, H, L, VD = 3, 2, 60, 5
    gen = torch.Generator().manual_seed(3)
    s = torch.randn(B, H, L, generator=gen, dtype=torch.float64) * 3
    v = torch.randn(B, H, L, VD, generator=gen, dtype=torch.float64)
    s[1, :, :L // world] = -float("inf")                 # sample 1: rank 0's positions all masked
    cp = CPShard(L, halo=1)
    sl = slice(cp.start, cp.start + cp.shard_len)
    lse_r = torch.logsumexp(s[..., sl], dim=-1)
    o_r = torch.einsum("bhl,bhlv->bhv", torch.exp(s[..., sl] - lse_r[..., None]).nan_to_num(0.0), v[:, :, sl])
    o_r[torch.isneginf(lse_r)] = float("nan")             # whatever the kernel leaves there
    lse_r[torch.isneginf(lse_r)] = float("inf")           # the kernels' "no mass" value
    o, lse = _cp_softmax_combine(o_r.reshape(B, H * VD).float(), lse_r.reshape(-1).float(), B, H, VD, cp)
    p = torch.softmax(s, dim=-1)
    o_ref = torch.einsum("bhl,bhlv->bhv", p, v).reshape(B, H * VD)
    ok = torch.allclose(o.double(), o_ref, atol=1e-5) and torch.allclose(lse.double(),
                                                                         torch.logsumexp(s, -1).reshape(-1), atol=1e-5)
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write("ok" if ok else "bad")
    dist.barrier()
    dist.destroy_process_group()


def test_cp_split_softmax_combine(tmp_path):
    """Paper-semantics CP attention: the shards' (o, logsumexp) merged by _cp_softmax_combine equal the
    softmax over all positions, also when one shard's positions are all masked for a sample."""
    world = 3
    mp.start_processes(_softmax_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       start_method="spawn", join=True)
    for r in range(world):
        assert (tmp_path / f"r{r}.txt").read_text() == "ok", r
