"""Parallelism over RCCL/xGMI: process-group bootstrap, bucketed all-reduce, sharded sampling,
ZeRO-1 sharded Adam (``zero``), context (sequence) parallelism over the residue axis
(``context_parallel``), the direct RCCL communicator of the gradient buckets (``rccl``) and the
DP-shared batch-axis softmax of the reference local head (``batch_softmax``).

Tensor/pipeline/expert parallelism are not provided: the reference has none and
the 16.8M-parameter model fits one MI355X many times over.
"""
from .dist import (DistInfo, init_distributed, get_info, is_main, barrier, all_reduce_max, all_reduce_mean_,
                   broadcast_module, destroy)
from .ddp import BucketedAllReduce
from . import batch_softmax
from .sampler import ShardedSampler
from .zero import ZeroFusedAdam
from .context_parallel import (ContextParallelProteinBERT, all_reduce_grads, cp_pretrain_loss, halo_exchange,
                               make_cp_groups)

__all__ = ["DistInfo", "init_distributed", "get_info", "is_main", "barrier", "all_reduce_max",
           "all_reduce_mean_", "broadcast_module", "destroy", "BucketedAllReduce", "ShardedSampler",
           "ContextParallelProteinBERT", "all_reduce_grads", "cp_pretrain_loss", "halo_exchange", "make_cp_groups",
           "ZeroFusedAdam", "batch_softmax"]
