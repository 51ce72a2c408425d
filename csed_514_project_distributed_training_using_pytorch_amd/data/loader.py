"""Device-resident batch loader (replaces DataLoader + workers + pin_memory).

Ref: src/train.py:25-41 (single-process loaders, shuffle=True) and
src/train_dist.py:40-45 (4 worker processes, pinned memory, sharded sampler).

On MI355X the whole uint8 dataset (47 MB for MNIST-train) lives in HBM.  A
batch is one ``gather_normalize`` kernel: it gathers the sampled rows, applies
ToTensor + Normalize((0.1307,), (0.3081,)) and writes the batch in the
compute dtype, plus the labels.  There are no worker processes, no pinned
host buffers and no host->device copies per batch.  On the CPU the same
iteration runs with stock tensor indexing (the test oracle).
"""
from __future__ import annotations

import math

import torch

from .mnist import MNIST_MEAN, MNIST_STD, MNISTData


class DeviceLoader:
    def __init__(self, data: MNISTData, batch_size: int, sampler=None, shuffle: bool = False,
                 device="cpu", dtype: torch.dtype = torch.float32, drop_last: bool = False,
                 mean: float = MNIST_MEAN, std: float = MNIST_STD, generator: torch.Generator | None = None):
        self.device = torch.device(device)
        self.data = data.to(self.device)
        self.dataset = self.data  # len(loader.dataset) like the reference
        self.batch_size = int(batch_size)
        self.sampler = sampler
        self.shuffle = shuffle
        self.dtype = dtype
        self.drop_last = drop_last
        self.mean, self.std = float(mean), float(std)
        self.generator = generator
        # optional (B, dtype) -> (x, target) buffers to gather into (e.g. a captured training
        # step's static inputs, engine/modular.py bind_loader) or None for fresh tensors
        self.into = None

    def _order(self) -> torch.Tensor:
        if self.sampler is not None:
            return self.sampler.indices()
        n = len(self.data)
        if self.shuffle:
            return torch.randperm(n, generator=self.generator)
        return torch.arange(n)

    def __len__(self) -> int:
        n = len(self.sampler) if self.sampler is not None else len(self.data)
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def batch(self, idx: torch.Tensor):
        """Gather + normalise the rows ``idx`` (device int64) -> (data [B,1,28,28], target [B])."""
        B = idx.numel()
        if self.device.type == "cuda":
            from ..ops import _native

            bufs = self.into(B, self.dtype) if self.into is not None else None
            if bufs is not None:
                out, lab = bufs
            else:
                out = torch.empty((B, 1, 28, 28), device=self.device, dtype=self.dtype)
                lab = torch.empty((B,), device=self.device, dtype=torch.long)
            _native.ops().gather_normalize(self.data.images, idx, None, B, self.mean, self.std, out, lab,
                                           self.data.labels)
            return out, lab
        x = self.data.images[idx].to(torch.float32).div_(255.0).sub_(self.mean).div_(self.std)
        return x.view(B, 1, 28, 28).to(self.dtype), self.data.labels[idx]

    def __iter__(self):
        order = self._order().to(self.device)
        n = order.numel()
        for s in range(0, n, self.batch_size):
            e = min(n, s + self.batch_size)
            if self.drop_last and e - s < self.batch_size:
                break
            yield self.batch(order[s:e])
