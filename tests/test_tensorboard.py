"""The dependency-free TensorBoard event writer (utils/tensorboard.py): CRC-32C test vector,
record framing and Event / Summary protobuf encoding read back, and pretrain(tensorboard_dir=...)
logging the reference's per-iteration loss / lr / time (ProteinBERT/utils.py:308-313) as scalars."""
import glob
import os

import torch

from proteinbert_pytorch_replication_amd.utils.tensorboard import (SummaryWriter, crc32c, masked_crc32c,
                                                                   read_scalars)


def test_crc32c_known_vectors():
    assert crc32c(b"123456789") == 0xE3069283          # CRC-32C check value
    assert crc32c(b"") == 0
    assert masked_crc32c(b"") == 0xA282EAD8


def test_scalars_round_trip(tmp_path):
    w = SummaryWriter(str(tmp_path))
    vals = [(1, "train/loss", 2.5), (1, "train/lr", 1e-4), (2, "train/loss", 2.25), (300000, "x", -3.0)]
    for step, tag, v in vals:
        w.add_scalar(tag, v, step)
    w.close()
    files = glob.glob(os.path.join(str(tmp_path), "events.out.tfevents.*"))
    assert len(files) == 1
    got = read_scalars(files[0])
    assert [(s, t) for s, t, _ in got] == [(s, t) for s, t, _ in vals]
    for (_, _, a), (_, _, b) in zip(got, vals):
        assert abs(a - b) <= 1e-7 * max(1.0, abs(b))
    with open(files[0], "rb") as f:
        head = f.read(64)
    assert b"brain.Event:2" in head


def test_pretrain_writes_tensorboard(tmp_path):
    from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
    from proteinbert_pytorch_replication_amd.models import ProteinBERT
    from proteinbert_pytorch_replication_amd.train.pretrain import pretrain
    torch.manual_seed(0)
    L, A = 32, 64
    m = ProteinBERT(sequences_length=L, num_annotations=A, local_dim=16, global_dim=32, key_dim=8, num_heads=2,
                    num_blocks=1)
    gen = SyntheticUniRefGO(L, A, 4, "cpu", seed=0)
    loader = [gen.next_batch() for _ in range(3)]
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    tb = str(tmp_path / "tb")
    mpath = str(tmp_path / "m.jsonl")
    res = pretrain(m, loader, opt, max_batch_iterations=3, save_path=str(tmp_path), tensorboard_dir=tb,
                   final_save=False, device="cpu", metrics_path=mpath)
    files = glob.glob(os.path.join(tb, "events.out.tfevents.*"))
    assert len(files) == 1
    got = read_scalars(files[0])
    losses = [v for s, t, v in got if t == "train/loss"]
    assert [s for s, t, _ in got if t == "train/loss"] == [1, 2, 3]
    assert all(abs(a - b) < 1e-5 * abs(b) for a, b in zip(losses, res["train_loss"]))
    assert {t for _, t, _ in got} == {"train/loss", "train/lr", "perf/step_time_s", "perf/seq_per_s"}
    # the JSONL record of each log interval: per-head losses summing to the total, tokens/s and MFU
    import json
    recs = [json.loads(x) for x in open(mpath)]
    assert len(recs) == 3
    for r in recs:
        assert abs(r["loss_local"] + r["loss_global"] - r["loss"]) < 1e-5 * max(1.0, abs(r["loss"]))
        assert r["tokens_per_s"] == r["seq_per_s"] * L and 0 < r["mfu"] < 1
