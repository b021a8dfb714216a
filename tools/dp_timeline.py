"""Data-parallel overlap evidence on ONE GPU: a 1-rank RCCL ("nccl") process group with the bucketed
all-reduce forced on (``BucketedAllReduce(force=True)``), so every 8 MB gradient bucket's collective
is issued on the communication stream while backward runs, exactly as on N ranks.

RCCL launches no kernel for a 1-rank all-reduce, so the timeline is taken with HIP events: one on the
main stream at the step start, one on the communication stream right before each bucket's
``all_reduce`` (it completes when the bucket's gradients are final: the comm stream waits for the main
and aux streams), one on the main stream after the last backward kernel and one after Adam.  A bucket
whose event lands before the backward end is a collective that runs under the backward on N ranks.

    python3 tools/dp_timeline.py --steps 6
(``--summarize trace.csv`` lists collective kernels of a multi-rank rocprofv3 kernel trace.)
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
    marks = []
    orig_ar = dist.all_reduce

    def all_reduce(t, *args, **kw):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(dev))          # the communication stream
        marks.append((ev, t.numel() * t.element_size()))
        return orig_ar(t, *args, **kw)

    dist.all_reduce = all_reduce
    orig_finish = ddp.finish

    def finish(*args, **kw):                               # called right after backward (+ aux join)
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(dev))
        marks.append((ev, -1))
        return orig_finish(*args, **kw)

    ddp.finish = finish
    orig_fs = ddp.finish_and_step

    def finish_and_step(*args, **kw):                      # overlapped optimizer (PretrainStep default)
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(dev))
        marks.append((ev, -1))
        return orig_fs(*args, **kw)

    ddp.finish_and_step = finish_and_step
    orig_range = opt.step_range
    ranges = []

    def step_range(s0, e0):                                # Adam launches: (start event, end event, elements)
        e_a = torch.cuda.Event(enable_timing=True)
        e_b = torch.cuda.Event(enable_timing=True)
        e_a.record(torch.cuda.current_stream(dev))
        orig_range(s0, e0)
        e_b.record(torch.cuda.current_stream(dev))
        ranges.append((e_a, e_b, e0 - s0))

    opt.step_range = step_range
    for i in range(a.steps):
        ranges.clear()
        marks.clear()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        loss = step(*gen.next_batch())
        t1.record()
        torch.cuda.synchronize()
        if i == a.steps - 1:
            total = t0.elapsed_time(t1)
            print(f"step {total:.3f} ms, {len(ddp.buckets)} buckets of <= {a.bucket_mb:g} MB, loss {float(loss):.4f}")
            bwd_end = next(t0.elapsed_time(ev) for ev, n in marks if n < 0)
            k = 0
            for ev, n in (x for x in marks if x[1] >= 0):
                t = t0.elapsed_time(ev)
                if n <= 8:      # the 4-byte group-wide non-finite flag (MAX), queued ahead of the last bucket
                    print(f"  non-finite flag (MAX all-reduce) enqueued at {t:7.3f} ms")
                    continue
                print(f"  bucket {k:2d}  {n / 2**20:6.2f} MB  gradients final at {t:7.3f} ms"
                      f"  ({'inside backward' if t < bwd_end - 1e-3 else 'after backward'})")
                k += 1
            print(f"  backward (+ aux streams) ends at {bwd_end:.3f} ms; Adam ends at {total:.3f} ms")
            last_ar = t0.elapsed_time([ev for ev, n in marks if n >= 0][-1])
            for e_a, e_b, n in ranges:
                print(f"  Adam over {n * 4 / 2**20:6.2f} MB of parameters: {t0.elapsed_time(e_a):7.3f} -> "
                      f"{t0.elapsed_time(e_b):7.3f} ms (last bucket's all-reduce enqueued at {last_ar:7.3f} ms)")
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
