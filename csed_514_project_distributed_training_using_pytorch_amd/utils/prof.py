"""Profiling helpers: ROCTx ranges and HIP-event step timers.

The reference only has wall-clock ``time.time() - t0`` prints (src/train.py:10,99,
src/train_dist.py:119,112).  Here:

* ``range(name)`` pushes/pops a ROCTx range (libroctx64 from the ROCm install
  or the one bundled with PyTorch) so rocprofv3 ``--marker-trace`` shows the
  step phases; it is a no-op when the library is absent.
* ``EventTimer`` brackets GPU work with HIP events (``torch.cuda.Event``) and
  reports device milliseconds without a host sync per step.
"""
from __future__ import annotations

import contextlib
import ctypes
import ctypes.util
import os
import time

import torch

_roctx = None


def _lib():
    global _roctx
    if _roctx is None:
        cands = [os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so"),
                 "/opt/rocm/lib/libroctx64.so", ctypes.util.find_library("roctx64")]
        _roctx = False
        for c in cands:
            if c and os.path.exists(c):
                try:
                    lib = ctypes.CDLL(c)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    _roctx = lib
                    break
                except OSError:
                    continue
    return _roctx or None


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    lib = _lib() if os.environ.get("CSED_ROCTX", "1") == "1" else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


class EventTimer:
    """Device-time stopwatch: ``start()`` / ``stop()`` record events, ``ms()`` syncs once."""

    def __init__(self, device=None):
        self.cuda = torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda")
        self._s = self._e = None
        self._t0 = self._t1 = 0.0

    def start(self):
        if self.cuda:  # both events made here: stop() inside a timed region only records
            self._s = torch.cuda.Event(enable_timing=True)
            self._e = torch.cuda.Event(enable_timing=True)
            self._e.record()  # creates the HIP event now; stop() records it again
            self._s.record()
        self._t0 = time.perf_counter()
        return self

    def stop(self):
        if self.cuda:
            self._e.record()
        self._t1 = time.perf_counter()
        return self

    def ms(self) -> float:
        if self.cuda and self._s is not None and self._e is not None:
            self._e.synchronize()
            return self._s.elapsed_time(self._e)
        return (self._t1 - self._t0) * 1e3
