"""MNIST storage: IDX reader/writer and a deterministic synthetic generator.

Replaces torchvision.datasets.MNIST (ref src/train.py:26-40,
src/train_dist.py:22-30), which is not available here.  Real MNIST is read
from the torchvision directory layout (``<root>/MNIST/raw/*-ubyte[.gz]``) or
a flat ``<root>/*-ubyte[.gz]``.  With no files (no network on this platform)
a synthetic, class-conditional 1x28x28 dataset of the same shape is
generated instead: it is learnable (each class has its own stroke template,
randomly shifted, scaled and noised), so loss curves are meaningful.

Everything is kept as raw ``uint8`` pixels; ToTensor + Normalize happens on
the device inside the batch-gather kernel (see data/loader.py).
"""
from __future__ import annotations

import gzip
import os
import struct
from dataclasses import dataclass
from pathlib import Path

import numpy as np
import torch

MNIST_MEAN = 0.1307
MNIST_STD = 0.3081
_FILES = {
    True: ("train-images-idx3-ubyte", "train-labels-idx1-ubyte"),
    False: ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte"),
}
_DTYPES = {0x08: np.uint8, 0x09: np.int8, 0x0B: np.dtype(">i2"), 0x0C: np.dtype(">i4"),
           0x0D: np.dtype(">f4"), 0x0E: np.dtype(">f8")}
_CODES = {np.dtype(np.uint8): 0x08, np.dtype(np.int8): 0x09}


def _open(path: Path):
    return gzip.open(path, "rb") if str(path).endswith(".gz") else open(path, "rb")


def read_idx(path) -> np.ndarray:
    """Parse an IDX file (optionally gzip-compressed) into a numpy array."""
    path = Path(path)
    with _open(path) as f:
        data = f.read()
    if len(data) < 4 or data[0] != 0 or data[1] != 0:
        raise ValueError(f"{path}: not an IDX file")
    code, ndim = data[2], data[3]
    if code not in _DTYPES:
        raise ValueError(f"{path}: unknown IDX dtype 0x{code:02x}")
    dims = struct.unpack(">" + "I" * ndim, data[4:4 + 4 * ndim])
    dt = np.dtype(_DTYPES[code])
    arr = np.frombuffer(data, dtype=dt, offset=4 + 4 * ndim, count=int(np.prod(dims)))
    return arr.reshape(dims).astype(dt.newbyteorder("=") if dt.byteorder == ">" else dt, copy=True)


def write_idx(path, arr: np.ndarray) -> None:
    arr = np.ascontiguousarray(arr)
    code = _CODES.get(arr.dtype)
    if code is None:
        raise ValueError("write_idx supports uint8/int8 arrays")
    header = bytes([0, 0, code, arr.ndim]) + struct.pack(">" + "I" * arr.ndim, *arr.shape)
    opener = gzip.open if str(path).endswith(".gz") else open
    with opener(path, "wb") as f:
        f.write(header + arr.tobytes())


@dataclass
class MNISTData:
    images: torch.Tensor  # uint8 [N, 28, 28]
    labels: torch.Tensor  # int64 [N]
    synthetic: bool = False

    def __len__(self) -> int:
        return int(self.images.shape[0])

    def to(self, device) -> "MNISTData":
        return MNISTData(self.images.to(device), self.labels.to(device), self.synthetic)


def _find(root: Path, name: str) -> Path | None:
    for d in (root / "MNIST" / "raw", root):
        for suffix in ("", ".gz"):
            p = d / (name + suffix)
            if p.exists():
                return p
    return None


def load_mnist(root, train: bool = True) -> MNISTData | None:
    """Real MNIST from ``root`` if its IDX files exist, else None."""
    root = Path(root)
    img_name, lab_name = _FILES[train]
    pi, pl = _find(root, img_name), _find(root, lab_name)
    if pi is None or pl is None:
        return None
    images = torch.from_numpy(read_idx(pi)).to(torch.uint8)
    labels = torch.from_numpy(read_idx(pl).astype(np.int64))
    if images.dim() != 3 or images.shape[0] != labels.shape[0]:
        raise ValueError(f"{root}: malformed MNIST files")
    return MNISTData(images, labels, synthetic=False)


def _templates(rng: np.random.Generator, classes: int) -> np.ndarray:
    """One smooth stroke template per class (float32 [classes, 28, 28] in [0,1])."""
    yy, xx = np.mgrid[0:28, 0:28].astype(np.float32)
    out = np.zeros((classes, 28, 28), np.float32)
    for c in range(classes):
        img = np.zeros((28, 28), np.float32)
        # a random polyline of 3-5 strokes inside the central 20x20 box
        pts = rng.uniform(6, 22, size=(rng.integers(4, 7), 2))
        for (y0, x0), (y1, x1) in zip(pts[:-1], pts[1:]):
            for t in np.linspace(0.0, 1.0, 24):
                cy, cx = y0 + t * (y1 - y0), x0 + t * (x1 - x0)
                img = np.maximum(img, np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / 2.2))
        out[c] = img / max(img.max(), 1e-6)
    return out


def synthetic_mnist(n: int, seed: int = 0, train: bool = True, classes: int = 10) -> MNISTData:
    """Deterministic, learnable MNIST-shaped data (uint8 1x28x28, labels 0..9)."""
    rng = np.random.default_rng(seed)
    tmpl = _templates(np.random.default_rng(12345), classes)  # same classes for train and test
    rng = np.random.default_rng(seed * 2 + (0 if train else 1) + 7)
    labels = rng.integers(0, classes, size=n).astype(np.int64)
    images = np.empty((n, 28, 28), np.uint8)
    chunk = 4096
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        m = e - s
        base = tmpl[labels[s:e]]
        dy = rng.integers(-2, 3, size=m)
        dx = rng.integers(-2, 3, size=m)
        amp = rng.uniform(0.7, 1.0, size=(m, 1, 1)).astype(np.float32)
        shifted = np.empty_like(base)
        for i in range(m):
            shifted[i] = np.roll(np.roll(base[i], dy[i], axis=0), dx[i], axis=1)
        noise = rng.normal(0.0, 0.08, size=base.shape).astype(np.float32)
        images[s:e] = np.clip((shifted * amp + noise) * 255.0, 0, 255).astype(np.uint8)
    return MNISTData(torch.from_numpy(images), torch.from_numpy(labels), synthetic=True)


def get_mnist(root=None, train: bool = True, synthetic: bool | None = None, n: int | None = None,
              seed: int = 0) -> MNISTData:
    """Real MNIST when available (and not ``synthetic=True``), otherwise synthetic data.

    ``n`` defaults to the real split sizes (60,000 train / 10,000 test).
    """
    root = Path(root if root is not None else os.path.join(os.getcwd(), "files"))
    if not synthetic:
        real = load_mnist(root, train)
        if real is not None:
            return real
        if synthetic is False:
            raise FileNotFoundError(f"MNIST IDX files not found under {root}")
    size = n if n is not None else (60000 if train else 10000)
    return synthetic_mnist(size, seed=seed, train=train)
