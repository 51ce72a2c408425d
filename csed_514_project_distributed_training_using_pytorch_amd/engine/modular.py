"""Per-op training engine: any nn.Module built from the csed ops, autograd, the
bucketed data-parallel reducer and the fused flat SGD.

This is the general path (every kernel is a separate HIP launch; the module
can be anything the op library supports).  ``Net`` additionally has the fused
two-launch engine in :mod:`.fused`.  Mirrors the reference's loops:
``train(epoch)`` / ``test()`` (ref src/train.py:69-104) and the DDP
``main()`` (ref src/train_dist.py:58-116).
"""
from __future__ import annotations

import torch

from .. import ops
from ..optim.sgd import FusedSGD
from ..parallel.ddp import DistributedDataParallel


class ModularTrainer:
    def __init__(self, model: torch.nn.Module, lr: float, momentum: float, ctx=None, loss: str = "nll",
                 bucket_cap_mb: float = 25.0, dampening: float = 0.0, weight_decay: float = 0.0,
                 nesterov: bool = False):
        self.ctx = ctx
        self.model = model
        self.distributed = ctx is not None and ctx.is_distributed
        params = list(model.parameters())
        if self.distributed:
            self.ddp = DistributedDataParallel(model, bucket_cap_mb=bucket_cap_mb)
            self.opt = FusedSGD(params, lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                nesterov=nesterov, flat=self.ddp.flat)
            self.forward = self.ddp
        else:
            self.ddp = None
            self.opt = FusedSGD(params, lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                nesterov=nesterov)
            self.forward = model
        if self.opt.on_gpu:
            ops.rng.default_state.device_step = self.opt.step_count  # graph-replay-safe dropout masks
        self.loss_name = loss

    def loss_fn(self, out, target):
        if self.loss_name == "ce":
            return ops.cross_entropy(out, target)  # nn.CrossEntropyLoss on log-probs (ref train_dist.py:67)
        return ops.nll_loss(out, target)

    def train_batch(self, x: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        """zero_grad -> forward -> loss -> backward (-> bucketed all-reduce) -> SGD. Returns the loss (device)."""
        self.model.train()
        self.opt.zero_grad()
        out = self.forward(x)
        loss = self.loss_fn(out, target)
        loss.backward()
        self.opt.step()
        return loss.detach()

    @torch.no_grad()
    def evaluate(self, loader) -> tuple[torch.Tensor, torch.Tensor, list]:
        """Summed NLL and correct count over ``loader`` (kept on device), plus per-batch mean losses."""
        self.model.eval()
        dev = next(self.model.parameters()).device
        total = torch.zeros((), device=dev)
        correct = torch.zeros((), device=dev, dtype=torch.long)
        batch_means = []
        for x, t in loader:
            out = self.model(x)
            total += ops.nll_loss(out, t, reduction="sum")
            batch_means.append(ops.nll_loss(out, t))
            correct += ops.accuracy_count(out, t)
        return total, correct, batch_means
