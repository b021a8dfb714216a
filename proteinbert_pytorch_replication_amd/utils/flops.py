"""Analytic training FLOPs of a ProteinBERT step (for the MFU field of the metrics).

Counts the multiply-adds of the matrix products (2 FLOP each) of reference ``modules.py``: the two
dilated convs, the local MLP, the attention value projection (and, unless ``useful_only``, the key
projection and the query, which reference semantics computes but whose softmax is over identical rows,
SURVEY A.2 Q1), the global MLP pair, the global->local vectors, the GO input layer and both heads.
Training = 3 x forward (backward = data + weight gradients).  Paper config at L = 512: 7.0 GFLOP useful,
7.6 GFLOP with the dead query/key path (BASELINE.md's torch FlopCounter figure of the reference graph,
8.84 GFLOP, also counts products this estimate leaves out).
"""
from __future__ import annotations

MI355X_BF16_DENSE_PEAK = 2.5e15      # FLOP/s, dense (no 2:4 sparsity)


def train_flops_per_sequence(config: dict, seq_len: int, useful_only: bool = True) -> float:
    L = seq_len
    C, G, A = config["local_dim"], config["global_dim"], config["num_annotations"]
    H, K = config["num_heads"], config["key_dim"]
    VD = G // H
    KS, V = config["conv_kernel_size"], config["vocab_size"]
    per_block = (2 * L * C * C * KS          # narrow + wide conv
                 + L * C * C                 # local MLP
                 + L * C * H * VD            # attention values
                 + 2 * G * G                 # global MLP pair
                 + G * C)                    # global -> local broadcast vector
    if not useful_only:
        per_block += L * C * H * K + G * H * K   # keys (per position) and queries (per sample)
    fwd = config["num_blocks"] * per_block + A * G + L * C * V + G * A
    return 3.0 * 2.0 * fwd


def mfu(flops_per_seq: float, seq_per_s: float, peak: float = MI355X_BF16_DENSE_PEAK, n_devices: int = 1) -> float:
    return flops_per_seq * seq_per_s / (peak * max(1, n_devices))
