"""Operator library: gfx950 HIP kernels exposed as differentiable PyTorch ops."""
from . import _native, rng
from .functional import (
    accuracy_count,
    compute_dtype,
    conv2d,
    conv2d_pool_relu,
    cross_entropy,
    dropout,
    dropout2d,
    dropout2d_scale,
    linear,
    linear_log_softmax_nll,
    mlp_head_nll,
    log_softmax,
    log_softmax_nll,
    max_pool2d_relu,
    nll_loss,
    set_compute_dtype,
    set_defer_wgrad_reduce,
    set_grad_destination,
)

__all__ = [
    "accuracy_count", "compute_dtype", "conv2d", "conv2d_pool_relu", "cross_entropy", "dropout",
    "dropout2d", "dropout2d_scale", "linear", "linear_log_softmax_nll", "mlp_head_nll", "log_softmax", "log_softmax_nll", "max_pool2d_relu", "nll_loss",
    "set_compute_dtype", "set_defer_wgrad_reduce", "set_grad_destination", "rng", "_native",
]
