"""Model summary table (the role ``torchinfo.summary`` plays in reference ``dummy_tests.py:120-125``).

``summary(model, col_names=("num_params", "trainable"), col_width=20, row_settings=("var_names",))``
returns a :class:`ModelStatistics` whose ``str()`` is a layer table; parameters that live outside
``nn.Module`` registration (none here - the attention heads are registered) are not counted, as in
torchinfo.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence

import torch.nn as nn


@dataclass
class ModelStatistics:
    rows: List[tuple]
    total_params: int
    trainable_params: int
    col_names: Sequence[str]
    col_width: int

    def __str__(self) -> str:
        w = self.col_width
        head = f"{'Layer (type (var_name))':60s}" + "".join(f"{c.replace('_', ' ').title():>{w}s}" for c in self.col_names)
        line = "=" * len(head)
        out = [line, head, line]
        for name, typ, depth, n, tr in self.rows:
            label = ("  " * depth + ("├─" if depth else "") + f"{typ} ({name})")[:60]
            cols = []
            for c in self.col_names:
                if c == "num_params":
                    cols.append(f"{n:>{w},}" if n else f"{'--':>{w}s}")
                elif c == "trainable":
                    cols.append(f"{tr:>{w}s}")
            out.append(f"{label:60s}" + "".join(cols))
        out += [line, f"Total params: {self.total_params:,}", f"Trainable params: {self.trainable_params:,}",
                f"Non-trainable params: {self.total_params - self.trainable_params:,}", line]
        return "\n".join(out)


def summary(model: nn.Module, col_names: Sequence[str] = ("num_params", "trainable"), col_width: int = 20,
            row_settings: Sequence[str] = ("var_names",), verbose: int = 0, max_depth: int = 3) -> ModelStatistics:
    rows = []

    def visit(mod: nn.Module, name: str, depth: int) -> None:
        own = list(mod.parameters(recurse=False))
        n = sum(p.numel() for p in mod.parameters())
        ps = list(mod.parameters())
        if not ps:
            tr = "--"
        elif all(p.requires_grad for p in ps):
            tr = "True"
        elif not any(p.requires_grad for p in ps):
            tr = "False"
        else:
            tr = "Partial"
        rows.append((name, type(mod).__name__, depth, n if (own or depth < max_depth) else n, tr))
        if depth < max_depth:
            for cname, child in mod.named_children():
                visit(child, cname, depth + 1)

    visit(model, type(model).__name__, 0)
    total = sum(p.numel() for p in model.parameters())
    trainable = sum(p.numel() for p in model.parameters() if p.requires_grad)
    stats = ModelStatistics(rows, total, trainable, tuple(col_names), col_width)
    if verbose:
        print(stats)
    return stats
