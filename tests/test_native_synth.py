"""Native synthetic-MNIST generator (csrc/data/synth_mnist.cpp via data/native_synth.py), CPU.

It stands in for the reference's dataset on disk (ref src/train_dist.py:22-30) in bench.py,
generating while ``import torch`` runs.  Checked here: determinism across thread counts (the
random stream is counter-based per sample), shapes / dtypes, a balanced label distribution,
pixel statistics close to data/mnist.py:synthetic_mnist's (same recipe, other random stream),
the shared stroke prototypes, and that it loads without torch.
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from csed_514_project_distributed_training_using_pytorch_amd import _build
from csed_514_project_distributed_training_using_pytorch_amd.data import native_synth, synthetic_mnist
from csed_514_project_distributed_training_using_pytorch_amd.data.mnist import _prototypes, native_synthetic_mnist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def lib():
    _build.build_data_lib(verbose=False)  # host g++ only: seconds
    native_synth._lib.cache_clear()
    assert native_synth.available()


def test_deterministic_across_thread_counts_and_splits():
    a_img, a_lab = native_synth.generate(3000, seed=0, train=True, threads=1)
    b_img, b_lab = native_synth.generate(3000, seed=0, train=True, threads=7)
    assert a_img.shape == (3000, 28, 28) and a_img.dtype == np.uint8 and a_lab.dtype == np.int64
    assert np.array_equal(a_img, b_img) and np.array_equal(a_lab, b_lab)
    # a prefix of a longer set is the shorter set (per-sample streams)
    c_img, c_lab = native_synth.generate(5000, seed=0, train=True, threads=3)
    assert np.array_equal(c_img[:3000], a_img) and np.array_equal(c_lab[:3000], a_lab)
    t_img, _ = native_synth.generate(3000, seed=0, train=False)
    s_img, _ = native_synth.generate(3000, seed=1, train=True)
    assert not np.array_equal(t_img, a_img) and not np.array_equal(s_img, a_img)


def test_distribution_close_to_torch_generator():
    img, lab = native_synth.generate(6000, seed=0, train=True)
    counts = np.bincount(lab, minlength=10)
    assert counts.min() > 500 and counts.max() < 700
    ref = synthetic_mnist(2000, seed=0)
    m, mr = img.astype(np.float64).mean(), ref.images.double().mean().item()
    assert abs(m - mr) < 0.1 * mr, (m, mr)
    # the fraction of bright (ink) pixels and the per-class mean images agree in shape
    ink, ink_r = (img > 128).mean(), (ref.images > 128).double().mean().item()
    assert abs(ink - ink_r) < 0.2 * ink_r, (ink, ink_r)
    for c in range(10):
        a = img[lab == c].astype(np.float64).mean(0).ravel()
        b = ref.images[ref.labels == c].double().mean(0).flatten().numpy()
        assert np.corrcoef(a, b)[0, 1] > 0.9, c


def test_shared_prototypes_and_mnistdata_wrapper():
    assert torch.equal(_prototypes(10), torch.from_numpy(native_synth.prototypes(10).copy()))
    d = native_synthetic_mnist(100, seed=3)
    assert d.synthetic and d.images.dtype == torch.uint8 and d.labels.dtype == torch.int64 and len(d) == 100


def test_loads_without_torch():
    code = ("import importlib.util, sys; "
            f"spec = importlib.util.spec_from_file_location('ns', {os.path.join(ROOT, 'csed_514_project_distributed_training_using_pytorch_amd', 'data', 'native_synth.py')!r}); "
            "ns = importlib.util.module_from_spec(spec); spec.loader.exec_module(ns); "
            "j = ns.Job(200, 50); (a, b), (c, d) = j.result(); "
            "assert a.shape == (200, 28, 28) and c.shape == (50, 28, 28); "
            "assert 'torch' not in sys.modules; print('ok')")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr
