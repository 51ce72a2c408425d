"""Data pipeline (IDX reader, synthetic MNIST, device loader) and DistributedSampler parity."""
import math

import numpy as np
import pytest
import torch
from torch.utils.data import DistributedSampler

from csed_514_project_distributed_training_using_pytorch_amd.data import (
    DeviceLoader, get_mnist, read_idx, synthetic_mnist, write_idx)
from csed_514_project_distributed_training_using_pytorch_amd.data.mnist import MNIST_MEAN, MNIST_STD, load_mnist
from csed_514_project_distributed_training_using_pytorch_amd.parallel.sampler import ShardSampler


@pytest.mark.parametrize("gz", [False, True])
def test_idx_roundtrip(tmp_path, gz):
    imgs = np.random.default_rng(0).integers(0, 256, size=(7, 28, 28), dtype=np.uint8)
    labs = np.arange(7, dtype=np.uint8)
    sfx = ".gz" if gz else ""
    write_idx(tmp_path / f"train-images-idx3-ubyte{sfx}", imgs)
    write_idx(tmp_path / f"train-labels-idx1-ubyte{sfx}", labs)
    assert np.array_equal(read_idx(tmp_path / f"train-images-idx3-ubyte{sfx}"), imgs)
    d = load_mnist(tmp_path, train=True)
    assert d is not None and not d.synthetic
    assert torch.equal(d.images, torch.from_numpy(imgs)) and d.labels.tolist() == list(range(7))
    assert load_mnist(tmp_path, train=False) is None


def test_torchvision_layout(tmp_path):
    raw = tmp_path / "MNIST" / "raw"
    raw.mkdir(parents=True)
    write_idx(raw / "t10k-images-idx3-ubyte", np.zeros((3, 28, 28), np.uint8))
    write_idx(raw / "t10k-labels-idx1-ubyte", np.array([1, 2, 3], np.uint8))
    d = get_mnist(tmp_path, train=False)
    assert len(d) == 3 and d.labels.tolist() == [1, 2, 3]


def test_idx_rejects_garbage(tmp_path):
    p = tmp_path / "x"
    p.write_bytes(b"\x01\x02\x03\x04junk")
    with pytest.raises(ValueError):
        read_idx(p)


def test_synthetic_is_deterministic_and_shaped():
    a = synthetic_mnist(300, seed=5)
    b = synthetic_mnist(300, seed=5)
    c = synthetic_mnist(300, seed=6)
    assert a.images.shape == (300, 28, 28) and a.images.dtype == torch.uint8
    assert a.labels.dtype == torch.int64 and int(a.labels.max()) <= 9
    assert torch.equal(a.images, b.images) and torch.equal(a.labels, b.labels)
    assert not torch.equal(a.images, c.images)
    # every class appears and classes are separable on average
    means = torch.stack([a.images[a.labels == k].float().mean(0) for k in range(10)])
    assert (torch.cdist(means.view(10, -1), means.view(10, -1)) + torch.eye(10) * 1e9).min() > 100


def test_get_mnist_falls_back_to_synthetic(tmp_path):
    d = get_mnist(tmp_path / "nothing", train=True, n=64)
    assert d.synthetic and len(d) == 64
    with pytest.raises(FileNotFoundError):
        get_mnist(tmp_path / "nothing", train=True, synthetic=False)


def test_cpu_loader_normalises_like_totensor_normalize():
    d = synthetic_mnist(100, seed=1)
    loader = DeviceLoader(d, 32, shuffle=False)
    batches = list(loader)
    assert len(batches) == len(loader) == 4 and batches[-1][0].shape == (4, 1, 28, 28)
    x, t = batches[0]
    ref = (d.images[:32].float() / 255.0 - MNIST_MEAN) / MNIST_STD
    torch.testing.assert_close(x.view(32, 28, 28), ref)
    assert torch.equal(t, d.labels[:32])
    assert len(DeviceLoader(d, 32, drop_last=True)) == 3


@pytest.mark.parametrize("n", [60000, 1001, 10])
@pytest.mark.parametrize("ws", [1, 2, 4, 8])
def test_shard_sampler_matches_distributed_sampler(n, ws):
    ds = list(range(n))
    for epoch in (0, 1, 5):
        for rank in range(ws):
            ref = DistributedSampler(ds, num_replicas=ws, rank=rank, shuffle=True, seed=42)
            ref.set_epoch(epoch)
            ours = ShardSampler(n, ws, rank, shuffle=True, seed=42)
            ours.set_epoch(epoch)
            assert ours.indices().tolist() == list(iter(ref))
            assert len(ours) == len(ref) == math.ceil(n / ws)


def test_shard_sampler_drop_last_and_no_shuffle():
    ds = list(range(103))
    for rank in range(4):
        ref = DistributedSampler(ds, num_replicas=4, rank=rank, shuffle=False, drop_last=True)
        ours = ShardSampler(103, 4, rank, shuffle=False, drop_last=True)
        assert ours.indices().tolist() == list(iter(ref))
    with pytest.raises(ValueError):
        ShardSampler(10, 2, 2)
