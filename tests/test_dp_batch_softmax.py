"""dp_batch_softmax (parallel/batch_softmax.py) on CPU, gloo, world_size 2: the reference local head's
softmax runs over the batch axis (ProteinBERT/modules.py:277-284), so data parallelism
only reproduces the single-process model when the ranks share that axis.  With the option on, DP=2 with
micro-batch b must equal ONE process with batch 2b -- the loss (mean over ranks of the per-rank means)
and the DP-averaged gradients; with it off the local-head gradients must differ (the test is sensitive).
SURVEY §4 item 5."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
from proteinbert_pytorch_replication_amd.models import ProteinBERT
from proteinbert_pytorch_replication_amd.parallel import batch_softmax

CFG = dict(sequences_length=32, num_annotations=40, local_dim=16, global_dim=32, key_dim=8, num_heads=4,
           num_blocks=2)
B = 3          # per rank


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _full_batch():
    return SyntheticUniRefGO(CFG["sequences_length"], CFG["num_annotations"], 2 * B, "cpu", seed=7,
                             use_kernel=False).next_batch()


def _slice(batch, r):
    return tuple({k: v[r * B:(r + 1) * B] for k, v in d.items()} for d in batch)


def _loss_and_grads(m, X, Y, W):
    from proteinbert_pytorch_replication_amd.train.losses import pretrain_loss_torch
    m.zero_grad(set_to_none=True)
    h, g = m.encode_torch(X["local"], X["global"], torch.float32)
    pl, pg = m.heads_torch(h, g)
    loss = pretrain_loss_torch(pl, pg, Y, {k: v.float() for k, v in W.items()})
    loss.backward()
    return loss.detach(), {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}


def _model():
    torch.manual_seed(0)
    return ProteinBERT(backend="torch", **CFG)


def _worker(rank, world, port, out_dir, on):
    import torch.distributed as dist
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        if on:
            batch_softmax.enable()
        assert batch_softmax.active() == on
        m = _model()
        loss, grads = _loss_and_grads(m, *_slice(_full_batch(), rank))
        dist.all_reduce(loss)
        for v in grads.values():
            dist.all_reduce(v)
        torch.save({"loss": loss / world, "grads": {k: v / world for k, v in grads.items()}},
                   os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        batch_softmax.disable()
        dist.destroy_process_group()


@pytest.mark.parametrize("on", [True, False])
def test_dp2_equals_single_process_batch_2b(tmp_path, on):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), on), nprocs=world, start_method="spawn",
                       join=True)
    res = torch.load(tmp_path / "r0.pt", weights_only=True)
    ref_loss, ref = _loss_and_grads(_model(), *_full_batch())
    head = "pretraining_local_output.0.weight"
    if not on:
        # per-micro-batch softmax: a different model (the local head's gradient moves by O(1) relative)
        err = ((res["grads"][head] - ref[head]).norm() / ref[head].norm()).item()
        assert err > 1e-3, err
        return
    assert abs(res["loss"].item() - ref_loss.item()) <= 1e-6 * abs(ref_loss.item())
    scale = max(v.norm().item() for v in ref.values())
    for k, v in ref.items():
        if k == "pretraining_local_output.0.bias":
            # exactly zero in exact arithmetic (softmax over the batch is shift-invariant per (l, v))
            assert res["grads"][k].abs().max().item() < 1e-6 * scale
            continue
        torch.testing.assert_close(res["grads"][k], v, rtol=1e-4, atol=1e-6 * scale, msg=k)


def test_inactive_without_process_group():
    assert not batch_softmax.active()
    z = torch.randn(4, 5, 6)
    torch.testing.assert_close(batch_softmax.softmax_over_batch(z), torch.softmax(z, dim=0))
