"""Loader for the in-tree native extension (``_C.so``, built by ``_build.py``).

The extension registers the ``torch.ops.csed.*`` operators (hand-written
gfx950 HIP kernels).  On a machine with a GPU every GPU op goes through these
kernels; if the shared object is missing or fails to load there, the ops
raise instead of silently running stock PyTorch kernels.
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

# CSED_NATIVE_SO: load another build of the extension (same-box A/B timing of two builds)
_SO = Path(os.environ.get("CSED_NATIVE_SO") or Path(__file__).resolve().parent.parent / "_C.so")
_lock = threading.Lock()
_loaded = False
_error: Exception | None = None

BF16, F16, F32 = 1, 2, 0
# compute dtype -> kernel code: 16-bit MFMA operands, or exact fp32 (v_mfma_f32_16x16x4_f32)
MFMA_CODE = {torch.bfloat16: BF16, torch.float16: F16, torch.float32: F32}


def so_path() -> Path:
    return _SO


def load(build_if_missing: bool | None = None) -> bool:
    """Load ``_C.so`` (optionally building it first).  Returns True on success."""
    global _loaded, _error
    with _lock:
        if _loaded:
            return True
        if build_if_missing is None:
            build_if_missing = os.environ.get("CSED_AUTOBUILD", "1") == "1"
        try:
            if not _SO.exists() and build_if_missing:
                from .. import _build

                _build.build(verbose=False)
            torch.ops.load_library(str(_SO))
            _loaded = True
            _error = None
        except Exception as e:  # pragma: no cover - exercised on broken installs
            _error = e
        return _loaded


def available() -> bool:
    return load()


def require() -> None:
    """Raise loudly when the HIP kernels are needed but not loadable."""
    if not load():
        raise RuntimeError(
            f"csed native extension could not be loaded from {_SO}: {_error!r}. "
            "Build it with `python -m csed_514_project_distributed_training_using_pytorch_amd._build`."
        )


def ops():
    require()
    return torch.ops.csed


def zeros(shape, dtype: torch.dtype = torch.float32, device=None) -> torch.Tensor:
    """torch.zeros on a GPU through the extension's own zero-fill kernel (lenet_fused.hip): torch's
    fill kernel sits in a large code object the HIP runtime loads at its first launch (5-60 ms on a
    fresh box, profiles/r6/epoch0.md), which the fused engine's bring-up should not pay."""
    t = torch.empty(shape, dtype=dtype, device=device)
    if t.device.type == "cuda":
        if t.numel():
            ops().lenet_zero_(t)
    else:
        t.zero_()
    return t


def zero_(t: torch.Tensor) -> torch.Tensor:
    """In-place zero of a contiguous tensor (see ``zeros``)."""
    if t.device.type == "cuda" and t.is_contiguous():
        if t.numel():
            ops().lenet_zero_(t)
    else:
        t.zero_()
    return t


def arange(n: int, device=None) -> torch.Tensor:
    """int64 0..n-1 (torch.arange's int64 case; see ``zeros``)."""
    t = torch.empty(int(n), dtype=torch.long, device=device)
    if t.device.type == "cuda":
        if t.numel():
            ops().lenet_iota_(t)
    else:
        torch.arange(int(n), out=t)
    return t
