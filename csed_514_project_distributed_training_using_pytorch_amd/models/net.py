"""The reference MNIST CNN (`Net`, ref src/model.py:4-22), MI355X-native.

Parameter names, shapes and default initialisation are those of the
reference (the layers are plain ``nn.Conv2d`` / ``nn.Linear`` parameter
containers, so ``torch.manual_seed(1); Net()`` yields bit-identical initial
weights and ``state_dict()`` files load into the reference model unchanged).

The GPU forward is five fused HIP kernels instead of ~15 ATen ops:

    conv1 + bias + maxpool2 + relu              (conv2d_pool_relu, fp32 input read directly)
    conv2 + bias + Dropout2d + maxpool2 + relu  (conv2d_pool_relu, mask drawn in the epilogue)
    fc1 + bias + relu + dropout                 (linear, act='relu_dropout')
    fc2 + bias                                  (linear, fp32 logits)
    log_softmax                                 (log_softmax)

(with targets: fc1 + relu + dropout + fc2 + log_softmax + NLL as ops.mlp_head_nll, one launch, the
loss returned)

The CPU forward is the reference forward verbatim in stock PyTorch (the fp32
oracle used by the tests).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops


class Net(nn.Module):
    """LeNet-style CNN: conv(1->10,k5) -> pool -> relu -> conv(10->20,k5) -> Dropout2d -> pool -> relu
    -> fc(320->50) -> relu -> dropout -> fc(50->10) -> log_softmax."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 10, kernel_size=5)
        self.conv2 = nn.Conv2d(10, 20, kernel_size=5)
        self.conv2_drop = nn.Dropout2d()
        self.fc1 = nn.Linear(320, 50)
        self.fc2 = nn.Linear(50, 10)

    # the modular engine may hand the targets to forward and get the mean NLL back: the classifier
    # head + log_softmax + NLL then run as ops.linear_log_softmax_nll (one backward launch for fc2
    # and the loss); without targets the module's output stays the log-probs
    fused_loss_head = True

    def forward(self, x: torch.Tensor, target: torch.Tensor | None = None) -> torch.Tensor:
        if not x.is_cuda:
            out = self.reference_forward(x)
            return out if target is None else F.nll_loss(out, target)
        # (the fp32 input is read and converted by conv1's staging: no cast launch)
        x = ops.conv2d_pool_relu(x, self.conv1.weight, self.conv1.bias)
        p2 = self.conv2_drop.p
        x = ops.conv2d_pool_relu(x, self.conv2.weight, self.conv2.bias,
                                 dropout2d_p=p2 if self.training else 0.0)  # Dropout2d drawn in-kernel
        x = x.view(-1, 320)
        act = "relu_dropout" if self.training else "relu"
        if target is not None:  # fc1 + relu + dropout + fc2 + log_softmax + NLL: one forward launch
            return ops.mlp_head_nll(x, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias, target,
                                    act=act, p=0.5)
        x = ops.linear(x, self.fc1.weight, self.fc1.bias, act=act, p=0.5)
        x = ops.linear(x, self.fc2.weight, self.fc2.bias, out_dtype=torch.float32)
        return ops.log_softmax(x, dim=1)

    def reference_forward(self, x: torch.Tensor) -> torch.Tensor:
        x = F.relu(F.max_pool2d(self.conv1(x), 2))
        x = F.relu(F.max_pool2d(self.conv2_drop(self.conv2(x)), 2))
        x = x.view(-1, 320)
        x = F.relu(self.fc1(x))
        x = F.dropout(x, training=self.training)
        x = self.fc2(x)
        return F.log_softmax(x, dim=1)


PARAM_SHAPES = [
    ("conv1.weight", (10, 1, 5, 5)),
    ("conv1.bias", (10,)),
    ("conv2.weight", (20, 10, 5, 5)),
    ("conv2.bias", (20,)),
    ("fc1.weight", (50, 320)),
    ("fc1.bias", (50,)),
    ("fc2.weight", (10, 50)),
    ("fc2.bias", (10,)),
]
N_PARAMS = 21840
