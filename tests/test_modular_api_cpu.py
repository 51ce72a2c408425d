"""CPU semantics of the modular engine's fused-op API (the stock-PyTorch oracle paths the GPU kernels
are held to in tests/test_modular_fusion_gpu.py):

* ops.linear_log_softmax_nll == nll_loss(log_softmax(linear(x)));
* ops.log_softmax_nll == nll_loss(log_softmax(z)) (and cross_entropy on log-probs is the same value);
* Net(x, target=t) == nll_loss(Net(x), t) with the same dropout draws;
* ModularTrainer.bind_loader leaves a CPU loader's batches unchanged.
"""
import torch
import torch.nn.functional as F

from csed_514_project_distributed_training_using_pytorch_amd import ops
from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist
from csed_514_project_distributed_training_using_pytorch_amd.data.loader import DeviceLoader
from csed_514_project_distributed_training_using_pytorch_amd.engine.modular import ModularTrainer
from csed_514_project_distributed_training_using_pytorch_amd.models import Net


def test_linear_log_softmax_nll_cpu():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(16, 50, generator=g, requires_grad=True)
    w = torch.randn(10, 50, generator=g, requires_grad=True)
    b = torch.randn(10, generator=g, requires_grad=True)
    t = torch.randint(0, 10, (16,), generator=g)
    for red in ("mean", "sum"):
        a = ops.linear_log_softmax_nll(x, w, b, t, red)
        r = F.nll_loss(F.log_softmax(F.linear(x, w, b), 1), t, reduction=red)
        torch.testing.assert_close(a, r)


def test_log_softmax_nll_and_cross_entropy_cpu():
    g = torch.Generator().manual_seed(1)
    z = torch.randn(32, 10, generator=g)
    t = torch.randint(0, 10, (32,), generator=g)
    ref = F.nll_loss(F.log_softmax(z, 1), t)
    torch.testing.assert_close(ops.log_softmax_nll(z, t), ref)
    # CrossEntropyLoss on log-probs (ref src/train_dist.py:67): log_softmax is idempotent
    torch.testing.assert_close(ops.cross_entropy(F.log_softmax(z, 1), t), ref)


def test_net_target_forward_cpu():
    torch.manual_seed(1)
    net = Net().train()
    x = torch.rand(8, 1, 28, 28)
    t = torch.randint(0, 10, (8,))
    torch.manual_seed(5)
    a = net(x, target=t)
    torch.manual_seed(5)
    b = F.nll_loss(net(x), t)
    torch.testing.assert_close(a, b)
    net.eval()
    assert net(x).shape == (8, 10)


def test_bind_loader_cpu_is_transparent():
    data = synthetic_mnist(64, seed=0)
    torch.manual_seed(0)
    tr = ModularTrainer(Net(), lr=0.01, momentum=0.5)
    dl = DeviceLoader(data, 16, shuffle=False)
    ref = [(x.clone(), t.clone()) for x, t in dl]
    tr.bind_loader(dl)
    got = list(dl)
    assert len(got) == len(ref)
    for (x, t), (xr, tr_) in zip(got, ref):
        assert torch.equal(x, xr) and torch.equal(t, tr_)
    loss = tr.train_batch(*got[0])
    assert torch.isfinite(loss)
