"""Data parallelism over RCCL/xGMI: process-group bootstrap, bucketed all-reduce, sharded sampling.

Tensor/pipeline/sequence/expert parallelism are not provided: the reference
has none and the 16.8M-parameter model plus L=4096 activations fit one
MI355X.
"""
from .dist import (DistInfo, init_distributed, get_info, is_main, barrier, all_reduce_max, all_reduce_mean_,
                   broadcast_module, destroy)
from .ddp import BucketedAllReduce
from .sampler import ShardedSampler

__all__ = ["DistInfo", "init_distributed", "get_info", "is_main", "barrier", "all_reduce_max",
           "all_reduce_mean_", "broadcast_module", "destroy", "BucketedAllReduce", "ShardedSampler"]
