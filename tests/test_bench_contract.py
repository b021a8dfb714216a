"""bench.py driver contract (README of the round driver): one JSON line from rank 0 with the metric /
config BASELINE.json names, whole-job value, max-over-ranks timing.  Rehearsed on the CPU with two gloo
ranks under torchrun (the RCCL path is the same code with backend "nccl" on a GPU node)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_lines(out: str):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


def test_bench_two_ranks_cpu_gloo():
    env = dict(os.environ, OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--batch", "2", "--seq-len", "32"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout                       # rank 0 only
    d = lines[0]
    assert KEYS <= set(d)
    assert d["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 4
    # whole-job aggregate: N * B * steps / (max-over-ranks seconds)
    assert abs(d["value"] - 2 * 2 * 1000.0 / d["ms_per_step"]) / d["value"] < 0.02


def test_bench_self_launches_ranks_cpu_gloo():
    """Plain ``python bench.py --gpus 2`` (no launcher): the script starts the two ranks itself and reports
    the real world size (the round driver may call it either way)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--batch", "2", "--seq-len", "32"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert d["n_gpus"] == 2 and d["world_size"] == 2 and d["backend"] == "gloo"
    assert d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 4
    assert d["dtype"] == "fp32" and "host" in d["data"]      # CPU rehearsal is labelled as such


def test_bench_rejects_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "1", "--warmup", "0",
           "--batch", "2", "--seq-len", "32"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
    assert not _json_lines(r.stdout)


def test_default_presets_size_batches_per_length():
    """Without --preset the bench takes the BASELINE preset of the mode / sequence length: ~1M tokens per
    GPU and step (cfg 2: 2048 x 512, cfg 3: 1024 x 1024, cfg 4: 256 x 4096, cfg 5 fine-tune: 2048 x 512)."""
    sys.path.insert(0, ROOT)
    import bench
    from proteinbert_pytorch_replication_amd.config import get_preset
    got = {k: get_preset(bench.default_preset(*k)) for k in [("pretrain", None), ("pretrain", 512),
                                                             ("pretrain", 1024), ("pretrain", 4096),
                                                             ("finetune", None)]}
    assert got[("pretrain", None)].name == got[("pretrain", 512)].name == "cfg2_paper_l512"
    assert got[("pretrain", 1024)].name == "cfg3_paper_l1024_dp8"
    assert got[("pretrain", 4096)].name == "cfg4_long_l4096_dp8"
    assert got[("finetune", None)].name == "cfg5_finetune_ss_l512_dp8"
    for (mode, L), cfg in got.items():
        tokens = cfg.train.batch_size * (L or cfg.model.sequences_length)
        assert tokens == 2 ** 20, (mode, L, tokens)
