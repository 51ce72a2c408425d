"""Per-op training engine: any nn.Module built from the csed ops, autograd, the
bucketed data-parallel reducer and the fused flat SGD.

This is the general path (every kernel is a separate HIP launch; the module
can be anything the op library supports).  ``Net`` additionally has the fused
two-launch engine in :mod:`.fused`.  Mirrors the reference's loops:
``train(epoch)`` / ``test()`` (ref src/train.py:69-104) and the DDP
``main()`` (ref src/train_dist.py:58-116).

A step is ``zero_grad -> forward -> loss -> backward (-> bucketed all-reduce on
the comm stream) -> SGD`` (ref src/train_dist.py:80-84).  On a GPU it runs as
ONE HIP-graph replay per step (``graph=True``, the default): the first batch
of each shape is captured once -- every op kernel, the reducer's RCCL calls on
their side stream, the SGD kernel -- and later batches are copied into the
captured input buffers and replayed, so the per-op path costs GPU time, not
~30 Python dispatches per step.  Two things make a replay the same step as an
eager call:

* gradients are written straight into the flat gradient buffer by the
  backward kernels (``ops.set_grad_destination``) and adopted by autograd
  without copies, with ``zero_grad`` setting ``.grad`` to None (no fill kernel);
* dropout masks are a pure function of (seed, device step counter, call index):
  the host offsets restart at every step, the optimizer's device step counter
  supplies the rest (``ops/rng.py``).

Graphs are not used where a collective cannot be captured (gloo) or on CPU.
"""
from __future__ import annotations

import sys

import torch

from .. import ops
from ..optim.sgd import FusedSGD
from ..parallel import comm
from ..parallel.ddp import DistributedDataParallel


class ModularTrainer:
    def __init__(self, model: torch.nn.Module, lr: float, momentum: float, ctx=None, loss: str = "nll",
                 bucket_cap_mb: float = 25.0, dampening: float = 0.0, weight_decay: float = 0.0,
                 nesterov: bool = False, graph: bool = True, overlap: bool = True):
        self.ctx = ctx
        self.model = model
        self.distributed = ctx is not None and ctx.is_distributed
        params = list(model.parameters())
        if self.distributed:
            self.ddp = DistributedDataParallel(model, bucket_cap_mb=bucket_cap_mb, overlap=overlap)
            self.opt = FusedSGD(params, lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                nesterov=nesterov, flat=self.ddp.flat)
            self.forward = self.ddp
        else:
            self.ddp = None
            self.opt = FusedSGD(params, lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                nesterov=nesterov)
            self.forward = model
        self.flat = self.opt.flat
        if self.opt.on_gpu:
            ops.rng.default_state.device_step = self.opt.step_count  # graph-replay-safe dropout masks
            for i, p in enumerate(self.flat.params):  # backward kernels write into the flat gradient
                ops.set_grad_destination(p, self.flat.grad_view(i))
        self.loss_name = loss
        self._fused_head = self.opt.on_gpu and loss in ("nll", "ce") and getattr(model, "fused_loss_head", False)
        gloo = self.distributed and getattr(ctx, "backend", None) != "nccl"
        self.use_graph = bool(graph) and self.opt.on_gpu and not gloo
        self._graphs: dict[tuple, tuple] = {}  # input shapes -> (graph, static x, static target, static loss)
        self._one: torch.Tensor | None = None

    def loss_fn(self, out, target):
        if self.loss_name == "ce":
            return ops.cross_entropy(out, target)  # nn.CrossEntropyLoss on log-probs (ref train_dist.py:67)
        return ops.nll_loss(out, target)

    def _forward_loss(self, x, target):
        """The model's output and the loss.  A model whose forward ends in log_softmax and takes
        the targets (``fused_loss_head``, e.g. ``Net``) returns the mean NLL itself, computed by its
        fused classifier-head + loss op: nll(log_softmax(z)) for 'nll', and for 'ce' the same value
        (CrossEntropyLoss on log-probs re-applies an idempotent log_softmax)."""
        if self._fused_head:
            return None, self.forward(x, target=target)
        out = self.forward(x)
        return out, self.loss_fn(out, target)

    def zero_grad(self) -> None:
        """set_to_none (torch's default): the next backward writes every gradient in place."""
        for p in self.flat.params:
            p.grad = None
        ops.functional.release_grad_buffers(self.flat.params)

    def _step(self, x: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        ops.rng.default_state.reset_offset()
        self.zero_grad()
        _, loss = self._forward_loss(x, target)
        if self._one is None or self._one.device != loss.device:
            self._one = torch.ones((), device=loss.device, dtype=loss.dtype)
        loss.backward(self._one)  # (a kept d loss / d loss: no fill kernel per step)
        self.opt.step()
        return loss.detach()

    def train_batch(self, x: torch.Tensor, target: torch.Tensor, clone_loss: bool = True) -> torch.Tensor:
        """zero_grad -> forward -> loss -> backward (-> bucketed all-reduce) -> SGD. Returns the loss (device).

        On a GPU the step is a graph replay (captured at the first batch of each shape); the
        returned loss is then a copy of the graph's output (``clone_loss=False``: the graph's own
        buffer, overwritten by the next step)."""
        self.model.train()
        if not self.use_graph:
            return self._step(x, target)
        key = self._graph_key(x, target)
        g = self._graphs.get(key)
        if g is None:
            g = self._capture(x, target)
            if g is None:
                return self._step(x, target)
        graph, sx, st, sloss = g
        if x.data_ptr() != sx.data_ptr():  # (a bound loader gathers straight into sx / st)
            sx.copy_(x, non_blocking=True)
        if target.data_ptr() != st.data_ptr():
            st.copy_(target, non_blocking=True)
        graph.replay()
        return sloss.clone() if clone_loss else sloss

    def _hyper(self) -> tuple:
        """The optimizer hyper-parameters a captured step bakes into its SGD launch: a change (an LR
        schedule, manual decay through ``opt.param_groups``) selects a new capture."""
        g = self.opt.param_groups[0]
        return (float(g["lr"]), float(g["momentum"]), float(g["dampening"]), float(g["weight_decay"]),
                bool(g["nesterov"]), float(self.opt.grad_scale))

    def _graph_key(self, x: torch.Tensor, target: torch.Tensor) -> tuple:
        return (tuple(x.shape), x.dtype, tuple(target.shape), self._hyper())

    def bind_loader(self, loader) -> None:
        """Let ``loader`` (data/loader.py DeviceLoader) gather each batch straight into the captured
        step's input buffers once a graph exists for its shape: no copy launches per step."""
        def into(B: int, dtype: torch.dtype):
            g = self._graphs.get(((B, 1, 28, 28), dtype, (B,), self._hyper())) if self.use_graph else None
            return (g[1], g[2]) if g is not None else None

        loader.into = into

    def _state(self) -> list[torch.Tensor]:
        return [self.flat.data, self.opt.momentum_flat, self.opt.step_count]

    def _capture(self, x: torch.Tensor, target: torch.Tensor):
        """Capture one step at these input shapes into a HIP graph (the engine state advanced by
        the capture's warm-up step is restored).  None (eager from then on) if capture fails."""
        dev = x.device
        sx, st = x.detach().clone(), target.detach().clone()
        state = self._state()
        saved = [t.clone() for t in state]
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        try:
            with torch.cuda.stream(s):
                self._step(sx, st)  # warm-up on the capture stream (lazy RCCL / allocator state)
            torch.cuda.current_stream(dev).wait_stream(s)
            torch.cuda.synchronize(dev)
            for t, v in zip(state, saved):
                t.copy_(v)
            torch.cuda.synchronize(dev)
            comm.quiesce()  # (no pending collective for the watchdog to query during the capture)
            graph = torch.cuda.CUDAGraph()
            # thread_local: the process group's watchdog thread may query earlier collectives'
            # events during the capture (see engine/fused.py _capture)
            with torch.cuda.graph(graph, stream=s, capture_error_mode="thread_local"):
                sloss = self._step(sx, st)
            torch.cuda.synchronize(dev)
        except Exception as e:  # an op or collective that cannot be captured: eager steps
            print(f"[csed] modular step capture failed ({e!r}); running eagerly", file=sys.stderr)
            torch.cuda.synchronize(dev)
            for t, v in zip(state, saved):
                t.copy_(v)
            self.use_graph = False
            return None
        g = (graph, sx, st, sloss)
        self._graphs[self._graph_key(x, target)] = g
        return g

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
