"""Model zoo: the reference LeNet (`Net`) plus generic building-block layers."""
from .layers import Conv2d, Dropout, Dropout2d, Linear
from .net import N_PARAMS, PARAM_SHAPES, Net

__all__ = ["Net", "PARAM_SHAPES", "N_PARAMS", "Conv2d", "Linear", "Dropout", "Dropout2d"]
