"""Distributed runtime: process groups (RCCL/gloo), bucketed DDP reducer, sharding, launcher."""
from .comm import DistContext, barrier, destroy, init_distributed, p2p_exchange
from .ddp import DDP, DistributedDataParallel, plan_buckets
from .sampler import ShardSampler

__all__ = ["DistContext", "init_distributed", "destroy", "barrier", "p2p_exchange", "DDP",
           "DistributedDataParallel", "plan_buckets", "ShardSampler"]
