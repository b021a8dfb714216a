"""Data-parallel overlap evidence on ONE GPU: a 1-rank RCCL ("nccl") process group with the bucketed
all-reduce forced on (``BucketedAllReduce(force=True)``), so every 8 MB gradient bucket's collective
is issued on the communication stream while backward runs, exactly as on N ranks.  Run it under
``rocprofv3 --kernel-trace`` and summarise with ``--summarize trace.csv``:

    rocprofv3 --kernel-trace --output-format csv -d out -- python3 tools/dp_timeline.py --steps 4
    python3 tools/dp_timeline.py --summarize out/.../kernel_trace.csv
"""
import argparse
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(a):
    import torch
    import torch.distributed as dist
    from proteinbert_pytorch_replication_amd.data import SyntheticUniRefGO
    from proteinbert_pytorch_replication_amd.models import ProteinBERT
    from proteinbert_pytorch_replication_amd.parallel.ddp import BucketedAllReduce
    from proteinbert_pytorch_replication_amd.train.optim import FusedAdam
    from proteinbert_pytorch_replication_amd.train.step import PretrainStep
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = ProteinBERT(sequences_length=512, num_annotations=8943, local_dim=128, global_dim=512, key_dim=64,
                    num_heads=4, num_blocks=6, device=dev, backend="hip")
    opt = FusedAdam(m.parameters(), lr=2e-4)
    ddp = BucketedAllReduce(opt.arena, bucket_mb=a.bucket_mb, force=True)
    step = PretrainStep(m, opt, ddp)
    gen = SyntheticUniRefGO(512, 8943, a.batch, dev, seed=1)
    for _ in range(a.steps):
        loss = step(*gen.next_batch())
    torch.cuda.synchronize()
    print(f"buckets {len(ddp.buckets)}  loss {float(loss):.4f}", flush=True)
    dist.destroy_process_group()


def summarize(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adam_flat" in r["Kernel_Name"]]
    seg = rows[idx[-2] + 1:idx[-1] + 1]          # the last full step (after one Adam, up to the next)
    t0 = int(seg[0]["Start_Timestamp"])
    comm = [r for r in seg if any(k in r["Kernel_Name"] for k in ("nccl", "Nccl", "rccl", "Rccl"))]
    qs = {}
    for r in seg:
        qs.setdefault(r["Queue_Id"], []).append(r)
    main = max(qs, key=lambda q: len(qs[q]))
    mk = qs[main]
    bwd0 = next((int(r["Start_Timestamp"]) for r in mk if "attn_bwd2" in r["Kernel_Name"]), t0)
    adam = int(seg[-1]["Start_Timestamp"])
    print(f"step span {(int(seg[-1]['End_Timestamp']) - t0) / 1e3:.1f} us; backward starts at "
          f"{(bwd0 - t0) / 1e3:.1f} us; Adam at {(adam - t0) / 1e3:.1f} us; {len(comm)} collective kernels")
    for r in comm:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        conc = [x["Kernel_Name"][:48] for x in mk if int(x["Start_Timestamp"]) < e and int(x["End_Timestamp"]) > s]
        print(f"  {(s - t0) / 1e3:8.1f} us  {(e - s) / 1e3:7.1f} us  q{r['Queue_Id']}  {r['Kernel_Name'][:40]:40s}"
              f"  beside: {conc[0] if conc else '-'}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--bucket-mb", type=float, default=8.0)
    ap.add_argument("--summarize", default=None)
    a = ap.parse_args()
    if a.summarize:
        summarize(a.summarize)
    else:
        run(a)
