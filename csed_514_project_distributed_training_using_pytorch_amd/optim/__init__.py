"""Optimizers: SGD-momentum as one fused HIP kernel over a flat buffer."""
from .sgd import FusedSGD

__all__ = ["FusedSGD"]
