"""Native synthetic-MNIST generation (``csrc/data/synth_mnist.cpp`` -> ``_csed_data.so``).

numpy + ctypes only -- no torch -- so ``bench.py`` and the CLIs can load this file on its own
(``importlib`` by path, before the package and before ``import torch``) and start generating the
70k-image set in a thread while the 1.4 s torch import runs: the ctypes call releases the GIL and
the generator spreads the samples over native threads.  This is the stand-in for the reference's
dataset on disk (ref src/train_dist.py:22-30 loads MNIST through torchvision).

The recipe is ``data/mnist.py:synthetic_mnist``'s with a counter-based random stream, so the
images differ from that function's (torch-generator) set but have the same distribution; the
stroke prototypes (``prototypes``) are shared by both.
"""
from __future__ import annotations

import ctypes
import functools
import os
import threading

import numpy as np

SYN_STYLES = 4  # stroke prototypes ("writing styles") per class
LIB_NAME = "_csed_data.so"


def lib_path() -> str:
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), LIB_NAME)


@functools.lru_cache(maxsize=1)
def _lib():
    path = lib_path()
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    fn = lib.csed_synth_mnist
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                   ctypes.c_void_p, ctypes.c_int]
    return lib


def available() -> bool:
    return _lib() is not None


def _raster(pts: np.ndarray, width: float) -> np.ndarray:
    """Anti-aliased polyline through ``pts`` ([k, 2] (y, x) in pixels) on a 28x28 canvas."""
    t = np.linspace(0.0, 1.0, 20, dtype=np.float32)[:, None]
    samples = np.concatenate([p0 + t * (p1 - p0) for p0, p1 in zip(pts[:-1], pts[1:])])  # [s, 2]
    yy, xx = np.mgrid[0:28, 0:28].astype(np.float32)
    d2 = (yy[None] - samples[:, 0, None, None]) ** 2 + (xx[None] - samples[:, 1, None, None]) ** 2
    img = np.exp(-d2 / (2.0 * width * width)).max(axis=0)
    return img / max(float(img.max()), 1e-6)


@functools.lru_cache(maxsize=4)
def prototypes(classes: int, styles: int = SYN_STYLES, seed: int = 12345) -> np.ndarray:
    """Per class, ``styles`` stroke prototypes (float32 [classes, styles, 28, 28] in [0, 1]).

    Each class has a core polyline of 4-6 points; its styles jitter every point by up to
    2.5 px and vary the stroke width, so a class is a mixture of related shapes rather than
    one template."""
    rng = np.random.default_rng(seed)
    out = np.zeros((classes, styles, 28, 28), np.float32)
    for c in range(classes):
        core = rng.uniform(6, 22, size=(rng.integers(4, 7), 2)).astype(np.float32)
        for s in range(styles):
            pts = np.clip(core + rng.uniform(-2.5, 2.5, size=core.shape).astype(np.float32), 4, 24)
            out[c, s] = _raster(pts, float(rng.uniform(0.9, 1.6)))
    out.setflags(write=False)
    return out


def _threads() -> int:
    n = os.cpu_count() or 4
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    # ranks of one node share its CPUs (torchrun / bench.py --gpus N export LOCAL_WORLD_SIZE)
    per_rank = n // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1))
    # (two CPUs left to the rank's HIP-context thread and main thread, which bring the runtime up
    # while the generator runs: 16 generator threads on a 16-CPU share slowed the context's
    # creation, profiles/r6/epoch0.md)
    return max(1, min(14, per_rank - 2))


def generate(n: int, seed: int = 0, train: bool = True, classes: int = 10,
             threads: int | None = None) -> tuple[np.ndarray, np.ndarray]:
    """(images uint8 [n, 28, 28], labels int64 [n]) from the native generator."""
    lib = _lib()
    if lib is None:
        raise RuntimeError(f"{lib_path()} is missing: build it with __graft_entry__.build()")
    protos = np.ascontiguousarray(prototypes(classes))
    images = np.empty((n, 28, 28), np.uint8)
    labels = np.empty((n,), np.int64)
    rc = lib.csed_synth_mnist(protos.ctypes.data, classes, n, seed, 1 if train else 0, images.ctypes.data,
                              labels.ctypes.data, threads or _threads())
    if rc != 0:
        raise RuntimeError(f"csed_synth_mnist failed ({rc})")
    return images, labels


class Job:
    """``generate`` for the train and test splits in a background thread (started at once)."""

    def __init__(self, n_train: int = 60000, n_test: int = 10000, seed: int = 0):
        self._out = None
        self._err = None
        self.elapsed_s = None  # the generator's own wall time
        self._t = threading.Thread(target=self._run, args=(n_train, n_test, seed), daemon=True)
        self._t.start()

    def _run(self, n_train, n_test, seed):
        import time

        t = time.perf_counter()
        try:
            self._out = (generate(n_train, seed, True), generate(n_test, seed, False))
        except BaseException as e:  # re-raised in result()
            self._err = e
        self.elapsed_s = time.perf_counter() - t

    def result(self):
        self._t.join()
        if self._err is not None:
            raise self._err
        return self._out
