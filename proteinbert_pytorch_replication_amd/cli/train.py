"""Training CLIs: ``pretrain`` and ``finetune`` (config presets + ``section.key=value`` overrides).

    python -m proteinbert_pytorch_replication_amd.cli pretrain --preset cfg2_paper_l512 \\
        train.max_batch_iterations=1000 data.source=store data.path=/data/uniref90.pbxds
    torchrun --nproc-per-node 8 -m proteinbert_pytorch_replication_amd.cli pretrain --preset ...

``data.source``: ``synthetic`` (on-device UniRef90-shaped batches), ``store`` (a ``.pbxds``/``.h5``
store or a directory of them, read by the native loader) or ``dataframe`` (``data.path`` = a CSV
with ``seq`` and space-separated ``annotations`` index columns).  The reference's own driver is
``dummy_tests.py`` (see :mod:`.dummy_tests`).

``finetune``: frozen (or full) encoder + per-residue head on synthetic secondary-structure data or a
CSV with ``seq`` and ``labels`` (one class character per residue, classes given by ``--classes``).
"""
from __future__ import annotations

import argparse
import json
import logging
import os
from typing import List, Optional

import torch

from ..config import RunConfig, apply_overrides, get_preset, load_yaml, PRESETS
from ..data import SyntheticUniRefGO, CorruptionParams
from ..models import ProteinBERT, ProteinBERTForTokenClassification, build_model
from ..utils import determinism
from ..parallel import dist as pdist


def _cfg(args) -> RunConfig:
    cfg = load_yaml(args.config) if args.config else get_preset(args.preset)
    return apply_overrides(cfg, args.overrides)


def _common(p: argparse.ArgumentParser) -> None:
    p.add_argument("--preset", default="cfg2_paper_l512", choices=sorted(PRESETS))
    p.add_argument("--config", default=None, help="YAML config (optionally with a `preset:` key)")
    p.add_argument("overrides", nargs="*", help="section.key=value overrides")


class _DataFrameAnnotations:
    """CSV -> reference DataFrame dataset rows (sequence, dense 0/1 annotation list)."""

    @staticmethod
    def load(path: str, num_annotations: int):
        import pandas as pd
        df = pd.read_csv(path)
        rows = []
        for seq, ann in zip(df["seq"], df.get("annotations", [""] * len(df))):
            dense = [0] * num_annotations
            for tok in str(ann).split():
                if tok and tok != "nan":
                    dense[int(tok)] = 1
            rows.append((seq, dense))
        return pd.DataFrame(rows)


def pretrain_main(argv: Optional[List[str]] = None) -> dict:
    ap = argparse.ArgumentParser(description="ProteinBERT pretraining (MI355X)")
    _common(ap)
    ap.add_argument("--resume", choices=["none", "latest"], default="latest")
    ap.add_argument("--metrics", default=None, help="JSONL metrics file (rank 0)")
    ap.add_argument("--tensorboard", default=None, help="TensorBoard event-file directory (rank 0)")
    ap.add_argument("--log-every", type=int, default=10)
    ap.add_argument("--async-checkpoint", action="store_true")
    ap.add_argument("--profile-steps", default=None, help="START[:COUNT] steps traced with torch.profiler")
    ap.add_argument("--profile-dir", default=None, help="trace output directory (default: save path)")
    ap.add_argument("--zero", action="store_true", help="ZeRO-1: shard the Adam moments over the DP ranks")
    a = ap.parse_args(argv)
    cfg = _cfg(a)
    logging.basicConfig(format="%(asctime)s [%(levelname)s]: %(message)s", level=logging.INFO)
    info = pdist.init_distributed(backend=cfg.dist.backend, timeout_s=cfg.dist.timeout_s)
    dev = info.device
    if cfg.kernel.deterministic:
        determinism.enable()
    if cfg.kernel.gelu != "fitted":
        from ..ops import _lib as _hiplib
        _hiplib.set_gelu(cfg.kernel.gelu)
    torch.manual_seed(cfg.train.seed)
    if cfg.data.lengths:
        # multi-length schedule: the LayerNorm affine is stored at the longest L and sliced per batch
        import dataclasses
        cfg.model = dataclasses.replace(cfg.model, sequences_length=max(int(x) for x in cfg.data.lengths),
                                        variable_length=True)
    model = build_model(cfg.model, device=dev, backend=determinism.backend_for(cfg.kernel.backend, cfg.model))
    B, L = cfg.train.batch_size, cfg.model.sequences_length
    corr = CorruptionParams(cfg.data.token_corruption_p, cfg.data.annotation_positive_p,
                            cfg.data.annotation_negative_p, cfg.data.blank_annotation_p)
    if cfg.data.source == "synthetic" and cfg.data.lengths:
        from ..data.synthetic import MultiLengthSynthetic
        loader = MultiLengthSynthetic(cfg.data.lengths, cfg.model.num_annotations, B, dev,
                                      seed=cfg.data.seed + 1000 * info.rank, min_length=cfg.data.min_length,
                                      density=cfg.data.annotation_density, corruption=corr)
    elif cfg.data.source == "synthetic":
        loader = SyntheticUniRefGO(L, cfg.model.num_annotations, B, dev, min_length=cfg.data.min_length,
                                   max_length=cfg.data.max_length, density=cfg.data.annotation_density,
                                   seed=cfg.data.seed + 1000 * info.rank, corruption=corr)
    elif cfg.data.source in ("store", "hdf5"):
        from ..train.dataloaders import create_pretrain_dataloaders
        loader = create_pretrain_dataloaders(cfg.data.path, B, recursive_dir=True, num_workers=cfg.data.num_workers,
                                             seq_max_length=L, device=dev, seed=cfg.data.seed)
    elif cfg.data.source == "dataframe":
        from torch.utils.data import DataLoader
        from ..data import UniRefGO_PretrainingDataset, collate_triples
        from ..parallel.sampler import ShardedSampler
        ds = UniRefGO_PretrainingDataset(_DataFrameAnnotations.load(cfg.data.path, cfg.model.num_annotations),
                                         seq_max_length=L)
        loader = DataLoader(ds, batch_size=B, sampler=ShardedSampler(len(ds), info.rank, info.world_size),
                            num_workers=cfg.data.num_workers, collate_fn=collate_triples, drop_last=True)
    else:
        raise ValueError(f"unknown data.source {cfg.data.source!r}")
    opt = torch.optim.Adam(model.parameters(), lr=cfg.optim.lr, betas=cfg.optim.betas, eps=cfg.optim.eps,
                           weight_decay=cfg.optim.weight_decay)
    from ..train.pretrain import pretrain
    res = pretrain(model, loader, opt, max_batch_iterations=cfg.train.max_batch_iterations,
                   save_path=cfg.train.save_path, nb_iterations_checkpoint=cfg.train.nb_iterations_checkpoint,
                   optim_scheduler_patience=cfg.optim.plateau_patience, warmup_duration=cfg.optim.warmup_duration,
                   device=dev, log_every=a.log_every, bucket_mb=cfg.dist.bucket_mb, compute_dtype=cfg.kernel.dtype,
                   grad_clip=cfg.optim.grad_clip, async_checkpoint=a.async_checkpoint, metrics_path=a.metrics,
                   tensorboard_dir=a.tensorboard,
                   resume=a.resume, profile_steps=a.profile_steps, profile_dir=a.profile_dir,
                   zero_optimizer=a.zero, comm_dtype=cfg.dist.comm_dtype,
                   dp_batch_softmax=cfg.dist.dp_batch_softmax)
    if info.is_main:
        print(json.dumps({"final_loss": res["train_loss"][-1] if res["train_loss"] else None,
                          "iterations": len(res["train_loss"]), "final_model": res.get("final_model_path")}))
    return res


def _ss_csv(path: str, L: int, classes: str):
    import pandas as pd
    from ..data.vocab import create_amino_acid_vocab, SOS_ID, EOS_ID
    v = create_amino_acid_vocab()
    cmap = {c: i for i, c in enumerate(classes)}
    df = pd.read_csv(path)
    toks, labs = [], []
    for seq, lab in zip(df["seq"], df["labels"]):
        seq, lab = str(seq)[: L - 2], str(lab)[: L - 2]
        t = [SOS_ID] + list(v.encode(seq)) + [EOS_ID]
        y = [-100] + [cmap.get(c, -100) for c in lab] + [-100]
        toks.append(t + [0] * (L - len(t)))
        labs.append(y + [-100] * (L - len(y)))
    return torch.utils.data.TensorDataset(torch.tensor(toks), torch.tensor(labs))


def finetune_main(argv: Optional[List[str]] = None) -> dict:
    ap = argparse.ArgumentParser(description="ProteinBERT fine-tuning: per-residue classification head")
    _common(ap)
    ap.add_argument("--pretrained", default=None, help="pretrained model/checkpoint (.pt) to start from")
    ap.add_argument("--train-csv", default=None)
    ap.add_argument("--test-csv", default=None)
    ap.add_argument("--classes", default="HEC", help="label alphabet (e.g. HEC or DSSP8 'HGIEBTSC')")
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--unfreeze", action="store_true", help="train the encoder as well")
    ap.add_argument("--synthetic-samples", type=int, default=2048)
    a = ap.parse_args(argv)
    cfg = _cfg(a)
    logging.basicConfig(format="%(asctime)s [%(levelname)s]: %(message)s", level=logging.INFO)
    info = pdist.init_distributed(backend=cfg.dist.backend)
    if cfg.kernel.deterministic:
        determinism.enable()
    if cfg.kernel.gelu != "fitted":
        from ..ops import _lib as _hiplib
        _hiplib.set_gelu(cfg.kernel.gelu)
    dev = info.device
    torch.manual_seed(cfg.train.seed)
    if a.pretrained:
        from ..train.checkpoint import load_model
        enc = load_model(a.pretrained, device=dev, backend=determinism.backend_for(cfg.kernel.backend, cfg.model))
    else:
        enc = build_model(cfg.model, device=dev, backend=determinism.backend_for(cfg.kernel.backend, cfg.model))
    L = enc.config["sequences_length"]
    model = ProteinBERTForTokenClassification(enc, n_classes=len(a.classes), freeze_encoder=not a.unfreeze)
    from torch.utils.data import DataLoader
    from ..data.synthetic import SyntheticSecondaryStructure
    from ..parallel.sampler import ShardedSampler
    if a.train_csv:
        train_ds = _ss_csv(a.train_csv, L, a.classes)
        test_ds = _ss_csv(a.test_csv, L, a.classes) if a.test_csv else None
    else:
        train_ds = SyntheticSecondaryStructure(a.synthetic_samples, L, len(a.classes), seed=cfg.train.seed)
        test_ds = SyntheticSecondaryStructure(max(64, a.synthetic_samples // 8), L, len(a.classes),
                                              seed=cfg.train.seed + 1)
    B = cfg.train.batch_size
    dl = DataLoader(train_ds, batch_size=B, sampler=ShardedSampler(len(train_ds), info.rank, info.world_size),
                    drop_last=True)
    tl = DataLoader(test_ds, batch_size=B) if test_ds is not None else None
    from ..train.optim import FusedAdam
    params = [p for p in model.parameters() if p.requires_grad]
    opt = FusedAdam(params, lr=a.lr)
    ddp = None
    if info.distributed:
        from ..parallel.ddp import BucketedAllReduce
        ddp = BucketedAllReduce(opt.arena, bucket_mb=cfg.dist.bucket_mb)
        ddp.broadcast_parameters(model)
        opt.grad_scale = 1.0 / info.world_size
    from ..train.finetune import finetune, token_accuracy
    res = finetune(model, dl, opt, epochs=a.epochs, test_dataloader=tl, metrics={"accuracy": token_accuracy()},
                   device=dev, ddp=ddp, log=print)
    if info.is_main:
        os.makedirs(cfg.train.save_path, exist_ok=True)
        path = os.path.join(cfg.train.save_path, "proteinbert_finetuned_head.pt")
        torch.save({k: v for k, v in model.state_dict().items() if not k.startswith("encoder.")}, path)
        print(json.dumps({"train_loss": res["train_loss"], "test_metrics": res["test_metrics"], "head": path}))
    return res
