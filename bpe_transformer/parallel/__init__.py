"""Distributed training over RCCL/xGMI: process groups and bucketed data parallelism."""

from .ddp import BucketedAllReduce
from .dist import DistInfo, all_reduce_max, all_reduce_mean_, barrier, cleanup, init_distributed

__all__ = ["BucketedAllReduce", "DistInfo", "all_reduce_max", "all_reduce_mean_", "barrier", "cleanup",
           "init_distributed"]
