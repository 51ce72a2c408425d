"""Drop-in ``torch.nn`` layers whose GPU path runs the gfx950 HIP kernels.

They subclass the stock modules, so parameter names, shapes, init and
``state_dict`` layout are unchanged; only ``forward`` is replaced.  Use them to
build other CNNs on the same kernels as :class:`Net`.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops


class Conv2d(nn.Conv2d):
    """Stride-1, symmetric-padding, dilation-1, groups-1 convolution (MFMA implicit GEMM)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        if self.stride != (1, 1) or self.dilation != (1, 1) or self.groups != 1:
            raise ValueError("csed Conv2d supports stride 1, dilation 1, groups 1")
        if isinstance(self.padding, str) or self.padding[0] != self.padding[1]:
            raise ValueError("csed Conv2d needs a symmetric integer padding")
        if self.padding_mode != "zeros":
            raise ValueError("csed Conv2d supports zero padding only")

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return ops.conv2d(x, self.weight, self.bias, padding=self.padding[0])


class Linear(nn.Linear):
    def __init__(self, in_features, out_features, bias=True, act: str = "none", device=None, dtype=None):
        super().__init__(in_features, out_features, bias, device, dtype)
        self.act = act

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return ops.linear(x, self.weight, self.bias, act=self.act)


class Dropout(nn.Dropout):
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return ops.dropout(x, self.p, self.training)


class Dropout2d(nn.Dropout2d):
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return ops.dropout2d(x, self.p, self.training)
