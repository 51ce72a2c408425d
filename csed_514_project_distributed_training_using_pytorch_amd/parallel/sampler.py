"""Rank sharding with exactly the index math of torch.utils.data.DistributedSampler.

The reference shards MNIST with ``DistributedSampler(num_replicas=world_size,
rank=rank, shuffle=True, seed=42)`` and calls ``set_epoch(i)`` every epoch
(ref src/train_dist.py:33-37,72).  This class reproduces the same indices
(``randperm(N, generator seeded seed+epoch)``, pad to a multiple of the world
size by wrapping, take ``indices[rank::world_size]``) but returns them as one
int64 tensor that can be uploaded to the device once per epoch, so the
training loop gathers batches on the GPU with no per-batch host work.
"""
from __future__ import annotations

import math

import torch


class ShardSampler:
    def __init__(self, dataset_len: int, num_replicas: int = 1, rank: int = 0, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False):
        if rank < 0 or rank >= num_replicas:
            raise ValueError(f"invalid rank {rank} for {num_replicas} replicas")
        self.n = int(dataset_len)
        self.num_replicas = int(num_replicas)
        self.rank = int(rank)
        self.shuffle = shuffle
        self.seed = int(seed)
        self.drop_last = drop_last
        self.epoch = 0
        if drop_last and self.n % self.num_replicas:
            self.num_samples = math.ceil((self.n - self.num_replicas) / self.num_replicas)
        else:
            self.num_samples = math.ceil(self.n / self.num_replicas)
        self.total_size = self.num_samples * self.num_replicas

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def global_indices(self) -> torch.Tensor:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g)
        else:
            idx = torch.arange(self.n)
        if not self.drop_last:
            pad = self.total_size - idx.numel()
            if pad > 0:
                reps = math.ceil(pad / idx.numel())
                idx = torch.cat([idx, idx.repeat(reps)[:pad]])
        else:
            idx = idx[: self.total_size]
        return idx

    def indices(self) -> torch.Tensor:
        """This rank's sample indices for the current epoch (int64, CPU)."""
        return self.global_indices()[self.rank:self.total_size:self.num_replicas].contiguous()

    def __iter__(self):
        return iter(self.indices().tolist())

    def __len__(self) -> int:
        return self.num_samples
