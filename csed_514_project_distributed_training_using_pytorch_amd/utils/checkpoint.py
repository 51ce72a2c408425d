"""Checkpoint files in the reference's format (ref src/train.py:84-85, src/train_dist.py:163-164).

* ``results/model.pth`` / ``model.pt``: ``Net.state_dict()`` -- the 8 fp32 CPU
  tensors ``conv1.weight ... fc2.bias`` (no ``module.`` prefix).
* ``results/optimizer.pth``: ``torch.optim.SGD.state_dict()`` layout.

Tensors are cloned to standalone CPU storages before ``torch.save`` (our
parameters are views into one flat device buffer), so the files are ordinary
PyTorch checkpoints that load into the reference ``Net``/``SGD`` unchanged.
Loading uses ``weights_only=True``.  Writes go to a temp file and are renamed,
so a concurrent reader never sees a torn file.  Resume (absent in the
reference) is :func:`load_checkpoint`.
"""
from __future__ import annotations

import os
from pathlib import Path

import torch


def _cpu_clone(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().to("cpu", copy=True).clone()
    if isinstance(obj, dict):
        return {k: _cpu_clone(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_cpu_clone(v) for v in obj)
    return obj


def _atomic_save(obj, path) -> None:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    tmp = path.with_name(path.name + f".tmp{os.getpid()}")
    torch.save(obj, tmp)
    os.replace(tmp, path)


def model_state(model: torch.nn.Module) -> dict:
    m = getattr(model, "module", model)
    return _cpu_clone(m.state_dict())


def save_model(model: torch.nn.Module, path) -> None:
    _atomic_save(model_state(model), path)


def save_optimizer(opt: torch.optim.Optimizer, path) -> None:
    _atomic_save(_cpu_clone(opt.state_dict()), path)


def save_checkpoint(model, opt, model_path="results/model.pth", opt_path="results/optimizer.pth") -> None:
    save_model(model, model_path)
    if opt is not None:
        save_optimizer(opt, opt_path)


def load_checkpoint(model, opt=None, model_path="results/model.pth", opt_path="results/optimizer.pth",
                    map_location="cpu") -> None:
    m = getattr(model, "module", model)
    sd = torch.load(model_path, map_location=map_location, weights_only=True)
    with torch.no_grad():
        own = m.state_dict()
        for k, v in sd.items():
            own[k].copy_(v)  # copy into existing (possibly flat-buffer) storage
    if opt is not None and opt_path and Path(opt_path).exists():
        opt.load_state_dict(torch.load(opt_path, map_location=map_location, weights_only=True))
