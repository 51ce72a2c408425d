"""Flat parameter / gradient storage.

All parameters of a model are re-homed into ONE contiguous fp32 buffer (and
their gradients into a second one) so the optimizer update is a single
multi-tensor kernel and the data-parallel gradient all-reduce is a single
collective over a contiguous range.  ``Net`` has 21,840 parameters =
87,360 bytes: the whole model is one bucket.
"""
from __future__ import annotations

from typing import Iterable

import torch


class FlatParams:
    def __init__(self, params: Iterable[torch.nn.Parameter]):
        self.params = [p for p in params]
        if not self.params:
            raise ValueError("no parameters")
        dev = self.params[0].device
        for p in self.params:
            if p.dtype != torch.float32:
                raise TypeError("FlatParams expects fp32 master parameters")
            if p.device != dev:
                raise ValueError("all parameters must live on one device")
        self.numels = [p.numel() for p in self.params]
        self.offsets = []
        off = 0
        for n in self.numels:
            self.offsets.append(off)
            off += n
        self.numel = off
        # pad the allocation to a multiple of 4 floats (16-B vector kernels)
        alloc = (off + 3) // 4 * 4
        from ..ops import _native  # (GPU: the extension's zero fill, not torch's -- see _native.zeros)

        self.data = _native.zeros(alloc, torch.float32, dev)
        self.grad = _native.zeros(alloc, torch.float32, dev)
        with torch.no_grad():
            for p, o, n in zip(self.params, self.offsets, self.numels):
                self.data[o:o + n].copy_(p.detach().reshape(-1))
                p.data = self.data[o:o + n].view_as(p)
        self.attach_grads()

    @property
    def device(self) -> torch.device:
        return self.data.device

    def view(self, flat: torch.Tensor, i: int) -> torch.Tensor:
        o, n = self.offsets[i], self.numels[i]
        return flat[o:o + n].view_as(self.params[i])

    def grad_view(self, i: int) -> torch.Tensor:
        return self.view(self.grad, i)

    def attach_grads(self) -> None:
        for i, p in enumerate(self.params):
            p.grad = self.grad_view(i)

    def gather_grads(self) -> None:
        """Make sure every param.grad is the flat view (copy in any stray grad tensor)."""
        for i, p in enumerate(self.params):
            v = self.grad_view(i)
            g = p.grad
            if g is None:
                v.zero_()
                p.grad = v
            elif g.data_ptr() != v.data_ptr():
                v.copy_(g)
                p.grad = v

    def zero_grad(self) -> None:
        self.grad.zero_()
        self.attach_grads()

    def grads_are_views(self) -> bool:
        return all(p.grad is not None and p.grad.data_ptr() == self.grad_view(i).data_ptr()
                   for i, p in enumerate(self.params))
