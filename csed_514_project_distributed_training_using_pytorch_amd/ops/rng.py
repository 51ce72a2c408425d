"""Philox stream bookkeeping for the dropout kernels.

Masks are a pure function of ``(seed, offset, element)`` (Philox4x32-10 in
``csrc/common.h``).  Every dropout call takes a fresh host ``offset``; when a
device step counter is attached (the optimizer's step tensor) its value is
added in the high bits on the device, so a captured HIP graph draws new masks
on every replay without any host involvement.
"""
from __future__ import annotations

import threading

import torch


class PhiloxState:
    def __init__(self, seed: int | None = None):
        self._seed = seed
        self._offset = 0
        self.device_step: torch.Tensor | None = None
        self._lock = threading.Lock()

    @property
    def seed(self) -> int:
        if self._seed is None:
            # follow torch.manual_seed() like the reference (ref src/train.py:21)
            self._seed = torch.initial_seed() & 0xFFFFFFFFFFFF
        return self._seed

    def manual_seed(self, seed: int) -> None:
        with self._lock:
            self._seed = int(seed) & 0xFFFFFFFFFFFF
            self._offset = 0

    def reset_offset(self) -> None:
        """Restart the host offsets (engine/modular.py calls it at every step start: with the
        device step counter in the high bits, masks are then a pure function of (seed, step,
        call index), identical between an eager step and a graph replay of it)."""
        with self._lock:
            self._offset = 0

    def next(self) -> tuple[int, int, torch.Tensor | None]:
        with self._lock:
            off = self._offset
            self._offset = (self._offset + 1) % (1 << 20)
        return self.seed, off, self.device_step


default_state = PhiloxState()


def manual_seed(seed: int) -> None:
    default_state.manual_seed(seed)


def philox_uniform_reference(seed: int, offset: int, idx):
    """NumPy reference of the device Philox draw (used by the numerics tests)."""
    import numpy as np

    idx = np.asarray(idx, dtype=np.uint64)
    M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
    W0, W1 = 0x9E3779B9, 0xBB67AE85
    mask = np.uint64(0xFFFFFFFF)
    x = idx & mask
    y = idx >> np.uint64(32)
    z = np.full_like(idx, np.uint64(offset & 0xFFFFFFFF))
    w = np.full_like(idx, np.uint64((offset >> 32) & 0xFFFFFFFF))
    k0 = seed & 0xFFFFFFFF
    k1 = (seed >> 32) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * x
        p1 = M1 * z
        hi0, lo0 = p0 >> np.uint64(32), p0 & mask
        hi1, lo1 = p1 >> np.uint64(32), p1 & mask
        nx = hi1 ^ y ^ np.uint64(k0)
        ny = lo1
        nz = hi0 ^ w ^ np.uint64(k1)
        nw = lo0
        x, y, z, w = nx, ny, nz, nw
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return (x >> np.uint64(8)).astype(np.float64) / 16777216.0
