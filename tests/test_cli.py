"""CLIs: pretrain (synthetic + store sources, resume), finetune, dummy_tests driver, summary."""
import json
import os

import numpy as np
import pytest
import torch

from proteinbert_pytorch_replication_amd.cli.__main__ import main as cli_main
from proteinbert_pytorch_replication_amd.cli.train import finetune_main, pretrain_main
from proteinbert_pytorch_replication_amd.models import ProteinBERT
from proteinbert_pytorch_replication_amd.utils.summary import summary

SMALL = ["model.sequences_length=32", "model.num_annotations=40", "model.local_dim=16", "model.global_dim=32",
         "model.key_dim=8", "model.num_blocks=1", "train.batch_size=4", "kernel.backend=torch", "kernel.dtype=fp32",
         "optim.warmup_duration=2", "train.nb_iterations_checkpoint=2"]


def test_pretrain_cli_synthetic_and_resume(tmp_path, capsys):
    args = ["--preset", "cfg1_cpu_smoke", *SMALL, f"train.save_path={tmp_path}", "train.max_batch_iterations=3",
            "--log-every", "1", "--metrics", str(tmp_path / "m.jsonl")]
    pretrain_main(args)
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert out["iterations"] == 3
    assert (tmp_path / "proteinbert_pretraining_checkpoint_2.pt").exists()
    assert len(open(tmp_path / "m.jsonl").read().splitlines()) == 3
    # resume=latest continues from iteration 2
    pretrain_main(["--preset", "cfg1_cpu_smoke", *SMALL, f"train.save_path={tmp_path}",
                   "train.max_batch_iterations=5"])
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert out["iterations"] == 3


def test_pretrain_cli_store_source(tmp_path, capsys):
    from proteinbert_pytorch_replication_amd.data.native_loader import native_loader_available
    from proteinbert_pytorch_replication_amd.data.store import ProteinStoreWriter
    if not native_loader_available():
        pytest.skip("host library not built")
    rng = np.random.default_rng(0)
    w = ProteinStoreWriter(str(tmp_path / "d.pbxds"), ["GO:%d" % i for i in range(40)])
    for i in range(20):
        w.append_mask("p%d" % i, "".join(rng.choice(list("ACDEFGHIKLMNPQRSTVWY"), 50)), rng.random(40) < 0.1)
    w.close()
    pretrain_main(["--preset", "cfg1_cpu_smoke", *SMALL, f"train.save_path={tmp_path}/ck",
                   "train.max_batch_iterations=7", "data.source=store", f"data.path={tmp_path}", "--resume", "none"])
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert out["iterations"] == 7          # crosses the 5-batch epoch boundary


def test_finetune_cli(tmp_path, capsys):
    csv = tmp_path / "ss.csv"
    csv.write_text("seq,labels\nACDEFGHIK,HHHEEECCC\nMKVLA,CCHHE\nWWWWWWWW,EEEECCCC\nAAAA,HHHH\n")
    finetune_main(["--preset", "cfg1_cpu_smoke", *SMALL, f"train.save_path={tmp_path}", "--train-csv", str(csv),
                   "--test-csv", str(csv), "--epochs", "2", "--classes", "HEC"])
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert len(out["train_loss"]) == 2 and os.path.exists(out["head"])
    head = torch.load(out["head"], weights_only=True)
    assert set(head) == {"head.weight", "head.bias", "global_head.weight"}


def test_dispatcher_and_dummy_tests(tmp_path, capsys):
    cli_main(["dummy-tests", "--iterations", "2", "--samples", "8", "--seq-len", "32", "--batch-size", "4",
              "--num-blocks", "1", "--annotations", "30", "--save-path", str(tmp_path), "--backend", "torch",
              "--device", "cpu", "--show-data"])
    out = capsys.readouterr().out
    assert "VOCAB:" in out and "Total params:" in out
    with pytest.raises(SystemExit):
        cli_main(["nope"])


def test_summary_counts_match_parameters():
    m = ProteinBERT(sequences_length=16, num_annotations=10, local_dim=8, global_dim=16, key_dim=4, num_heads=2,
                    num_blocks=1, device="cpu")
    s = summary(m)
    assert s.total_params == sum(p.numel() for p in m.parameters())
    assert "Total params" in str(s)


def test_task_splitting(monkeypatch):
    """U3 task-splitting helpers (reference shared_utils/util.py:436-505); the SLURM array id is read from
    the environment (U4's job-array helper itself is not needed)."""
    import argparse
    from proteinbert_pytorch_replication_amd.utils.cli_types import (add_parser_task_arguments,
                                                                     determine_parser_task_details)
    p = argparse.ArgumentParser()
    add_parser_task_arguments(p)
    assert determine_parser_task_details(p.parse_args(["--task-index", "2", "--total-tasks", "4"])) == (2, 4)
    for k in ("SLURM_ARRAY_TASK_ID", "TASK_ID_OFFSET", "TOTAL_TASKS"):
        monkeypatch.delenv(k, raising=False)
    assert determine_parser_task_details(p.parse_args([])) == (0, 1)
    monkeypatch.setenv("SLURM_ARRAY_TASK_ID", "3")
    monkeypatch.setenv("TASK_ID_OFFSET", "2")
    monkeypatch.setenv("TOTAL_TASKS", "40")
    assert determine_parser_task_details(p.parse_args([])) == (5, 40)
    with pytest.raises(ValueError):
        determine_parser_task_details(p.parse_args(["--task-index", "5", "--total-tasks", "4"]))
