"""Data-parallel gradient reducer (replaces torch DDP's C++ Reducer, ref src/train_dist.py:63).

Design for MI355X + RCCL over xGMI:

* **Flat storage.**  Parameters and gradients are re-homed into one flat fp32
  buffer each (``utils.flat.FlatParams``); a bucket is a contiguous slice of
  the flat gradient, so an all-reduce needs no copy-in / copy-out.
* **Buckets in reverse parameter order.**  Backward produces gradients from the
  last layer to the first, so buckets are cut from the end of the parameter
  list.  A bucket's all-reduce is launched (on a dedicated comm stream, after
  an event join with the compute stream) as soon as its last gradient has been
  accumulated, so it overlaps the remaining backward kernels.
* **Bucket size for xGMI.**  Each MI355X has 7 point-to-point xGMI links (~153
  GB/s each); a ring all-reduce of S bytes moves 2(N-1)/N*S per GPU and for
  S below a few hundred KB is latency-bound (14 dependent hops at N=8), so
  splitting a small model into many buckets only adds launches.  The default
  cap (``bucket_cap_mb``) therefore keeps whole layers together, and models the
  size of ``Net`` (87 KB) fit in one or two buckets.  ``plan_buckets`` exposes
  the cut so it can be tuned per model.
* **Init sync.**  Rank 0's parameters are broadcast once in one coalesced
  collective over the flat buffer (the reference's DDP constructor broadcast).
* **Averaging.**  RCCL reduces with ``ReduceOp.AVG`` (no separate divide
  kernel); gloo (CPU tests) sums then divides.

``no_sync()`` skips communication for gradient accumulation.
"""
from __future__ import annotations

import contextlib
from typing import Sequence

import torch
import torch.distributed as dist
import torch.nn as nn

from ..utils.flat import FlatParams


def plan_buckets(numels: Sequence[int], cap_elems: int) -> list[list[int]]:
    """Group parameter indices into buckets, walking from the LAST parameter.

    A bucket is closed once adding the next parameter would exceed ``cap_elems``
    (a single oversized parameter gets its own bucket).  Returned buckets list
    parameter indices in ascending order; bucket 0 holds the last parameters.
    """
    buckets: list[list[int]] = []
    cur: list[int] = []
    size = 0
    for i in reversed(range(len(numels))):
        n = numels[i]
        if cur and size + n > cap_elems:
            buckets.append(sorted(cur))
            cur, size = [], 0
        cur.append(i)
        size += n
    if cur:
        buckets.append(sorted(cur))
    return buckets


class _Bucket:
    def __init__(self, idx: list[int], flat: FlatParams):
        self.params = idx
        self.start = flat.offsets[idx[0]]
        last = idx[-1]
        self.end = flat.offsets[last] + flat.numels[last]
        self.pending = len(idx)
        self.launched = False
        self.work = None

    def view(self, flat: FlatParams) -> torch.Tensor:
        return flat.grad[self.start:self.end]


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, process_group=None, bucket_cap_mb: float = 25.0,
                 flat: FlatParams | None = None, broadcast_init: bool = True, overlap: bool = True):
        super().__init__()
        self.module = module
        self.pg = process_group
        self.world_size = dist.get_world_size(process_group) if dist.is_initialized() else 1
        params = [p for p in module.parameters() if p.requires_grad]
        self.flat = flat if flat is not None else FlatParams(params)
        self.backend = dist.get_backend(process_group) if dist.is_initialized() else None
        self.device = self.flat.device
        if broadcast_init and self.world_size > 1:
            dist.broadcast(self.flat.data, src=0, group=process_group)
        cap = max(1, int(bucket_cap_mb * 1024 * 1024 / 4))
        self.buckets = [_Bucket(b, self.flat) for b in plan_buckets(self.flat.numels, cap)]
        self._bucket_of = {}
        for bi, b in enumerate(self.buckets):
            for i in b.params:
                self._bucket_of[i] = bi
        self.overlap = overlap
        self._sync = True
        self._armed = False
        self._comm_stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self._hooks = []
        for i, p in enumerate(self.flat.params):
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))

    # ------------------------------------------------------------------ api
    def forward(self, *args, **kwargs):
        self._reset()
        return self.module(*args, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        prev = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = prev

    def bucket_sizes_bytes(self) -> list[int]:
        return [(b.end - b.start) * 4 for b in self.buckets]

    # ------------------------------------------------------------- internals
    def _reset(self) -> None:
        for b in self.buckets:
            b.pending = len(b.params)
            b.launched = False
            b.work = None
        self._armed = False

    def _make_hook(self, i: int):
        def hook(p: torch.Tensor) -> None:
            if not self._sync or self.world_size == 1:
                return
            v = self.flat.grad_view(i)
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                # AccumulateGrad produced a fresh tensor (grads were set to None): adopt it
                v.copy_(p.grad if p.grad is not None else torch.zeros_like(v))
                p.grad = v
            if not self._armed:
                self._armed = True
                torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
            b = self.buckets[self._bucket_of[i]]
            b.pending -= 1
            if b.pending == 0 and self.overlap:
                self._launch(b)

        return hook

    def _launch(self, b: _Bucket) -> None:
        if b.launched:
            return
        b.launched = True
        view = b.view(self.flat)
        if self.backend == "nccl":
            cs = self._comm_stream
            cs.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(cs):
                b.work = dist.all_reduce(view, op=dist.ReduceOp.AVG, group=self.pg, async_op=True)
        else:
            b.work = dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)

    def _finalize(self) -> None:
        for b in self.buckets:
            if not b.launched:
                self._launch(b)
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                if self.backend != "nccl":
                    b.view(self.flat).div_(self.world_size)
        if self._comm_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._comm_stream)
        self._armed = False


DDP = DistributedDataParallel
