"""SGD with momentum as ONE fused HIP kernel over a flat parameter buffer.

Drop-in for ``torch.optim.SGD(params, lr, momentum)`` (ref src/train.py:60-61,
src/train_dist.py:66): same update rule (dampening, weight decay, Nesterov),
same ``param_groups`` and the same ``state_dict()`` layout
(``state[i]['momentum_buffer']``), so ``results/optimizer.pth`` files are
interchangeable with stock PyTorch.

On the GPU the stock non-foreach SGD issues ~3 launches per parameter tensor
(24 for Net); here it is one launch over 21,840 floats.  The "first step"
flag lives on the device (a step counter bumped by the kernel's last block),
so the update is capturable in a HIP graph and replayable.
"""
from __future__ import annotations

import torch

from ..ops import _native
from ..utils.flat import FlatParams


class FusedSGD(torch.optim.SGD):
    def __init__(self, params, lr: float = 0.01, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, flat: FlatParams | None = None):
        params = list(params)
        super().__init__(params, lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                         nesterov=nesterov)
        if len(self.param_groups) != 1:
            raise ValueError("FusedSGD supports a single parameter group")
        plist = self.param_groups[0]["params"]
        self.flat = flat if flat is not None else FlatParams(plist)
        if [id(p) for p in self.flat.params] != [id(p) for p in plist]:
            raise ValueError("flat buffer parameters must match the optimizer parameters (same order)")
        dev = self.flat.device
        self.momentum_flat = torch.zeros_like(self.flat.data)
        self.step_count = torch.zeros(1, dtype=torch.long, device=dev)
        self._ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        self.grad_scale = 1.0

    @property
    def on_gpu(self) -> bool:
        return self.flat.device.type == "cuda"

    def zero_grad(self, set_to_none: bool = True) -> None:  # noqa: D401 - torch signature
        """Zero the flat gradient in one fill; grads stay views of the flat buffer."""
        self.flat.zero_grad()

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        g = self.param_groups[0]
        self.flat.gather_grads()
        if self.on_gpu:
            _native.ops().sgd_flat(self.flat.data, self.flat.grad, self.momentum_flat, float(g["lr"]),
                                   float(g["momentum"]), float(g["dampening"]), float(g["weight_decay"]),
                                   bool(g["nesterov"]), float(self.grad_scale), self.step_count, self._ticket)
        else:
            self._cpu_step(g)
        return loss

    def _cpu_step(self, g) -> None:
        lr, m, damp, wd, nest = g["lr"], g["momentum"], g["dampening"], g["weight_decay"], g["nesterov"]
        first = int(self.step_count.item()) == 0
        p, d, buf = self.flat.data, self.flat.grad * self.grad_scale, self.momentum_flat
        if wd:
            d = d + wd * p
        if m:
            if first:
                buf.copy_(d)
            else:
                buf.mul_(m).add_(d, alpha=1 - damp)
            d = d + m * buf if nest else buf
        p.add_(d, alpha=-lr)
        self.step_count += 1

    # ---- torch.optim.SGD-compatible state dict -------------------------------------------------
    def state_dict(self):
        if int(self.step_count.item()) > 0 and self.param_groups[0]["momentum"] != 0:
            for i, p in enumerate(self.flat.params):
                self.state[p]["momentum_buffer"] = self.flat.view(self.momentum_flat, i).detach().clone()
        sd = super().state_dict()
        return sd

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        have = False
        with torch.no_grad():
            for i, p in enumerate(self.flat.params):
                st = self.state.get(p, {})
                mb = st.get("momentum_buffer")
                if mb is not None:
                    self.flat.view(self.momentum_flat, i).copy_(mb)
                    have = True
        self.step_count.fill_(1 if have else 0)
