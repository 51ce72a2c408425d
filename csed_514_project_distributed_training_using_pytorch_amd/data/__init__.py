"""Data: MNIST IDX / synthetic storage and the device-resident loader."""
from .loader import DeviceLoader
from .mnist import MNIST_MEAN, MNIST_STD, MNISTData, get_mnist, load_mnist, read_idx, synthetic_mnist, write_idx

__all__ = ["DeviceLoader", "MNISTData", "get_mnist", "load_mnist", "read_idx", "write_idx", "synthetic_mnist",
           "MNIST_MEAN", "MNIST_STD"]
