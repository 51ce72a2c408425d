"""Net contract (names, shapes, init, forward) and the fused SGD optimizer on CPU."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from csed_514_project_distributed_training_using_pytorch_amd.models import N_PARAMS, PARAM_SHAPES, Net
from csed_514_project_distributed_training_using_pytorch_amd.optim import FusedSGD
from csed_514_project_distributed_training_using_pytorch_amd.utils import checkpoint
from csed_514_project_distributed_training_using_pytorch_amd.utils.flat import FlatParams


def _plain_lenet():
    """The reference architecture assembled from stock layers (independent oracle)."""
    m = nn.Module()
    m.conv1 = nn.Conv2d(1, 10, kernel_size=5)
    m.conv2 = nn.Conv2d(10, 20, kernel_size=5)
    m.conv2_drop = nn.Dropout2d()
    m.fc1 = nn.Linear(320, 50)
    m.fc2 = nn.Linear(50, 10)
    return m


def test_param_names_shapes_and_count():
    net = Net()
    sd = net.state_dict()
    assert [(k, tuple(v.shape)) for k, v in sd.items()] == PARAM_SHAPES
    assert sum(p.numel() for p in net.parameters()) == N_PARAMS == 21840


def test_seeded_init_matches_stock_layers():
    torch.manual_seed(1)
    a = Net()
    torch.manual_seed(1)
    b = _plain_lenet()
    for (k, v), (k2, v2) in zip(a.state_dict().items(), b.state_dict().items()):
        assert k == k2 and torch.equal(v, v2)


def test_cpu_forward_is_reference_forward():
    torch.manual_seed(0)
    net = Net().eval()
    x = torch.randn(5, 1, 28, 28)
    out = net(x)
    y = F.relu(F.max_pool2d(net.conv1(x), 2))
    y = F.relu(F.max_pool2d(net.conv2(y), 2)).view(-1, 320)
    y = net.fc2(F.relu(net.fc1(y)))
    torch.testing.assert_close(out, F.log_softmax(y, 1))
    assert torch.allclose(out.exp().sum(1), torch.ones(5))


@pytest.mark.parametrize("kw", [dict(lr=0.02, momentum=0.5), dict(lr=0.01, momentum=0.9, nesterov=True),
                                dict(lr=0.05, momentum=0.5, dampening=0.1, weight_decay=1e-3),
                                dict(lr=0.1, momentum=0.0)])
def test_fused_sgd_cpu_matches_torch(kw):
    torch.manual_seed(2)
    a = Net()
    b = copy.deepcopy(a)
    oa = FusedSGD(a.parameters(), **kw)
    ob = torch.optim.SGD(b.parameters(), **kw)
    for _ in range(4):
        x = torch.randn(8, 1, 28, 28)
        t = torch.randint(0, 10, (8,))
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            F.nll_loss(m.eval()(x), t).backward()
            o.step()
    for p, q in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-6, atol=1e-7)


def test_fused_sgd_state_dict_interop(tmp_path):
    torch.manual_seed(3)
    a = Net()
    oa = FusedSGD(a.parameters(), lr=0.01, momentum=0.5)
    x = torch.randn(4, 1, 28, 28)
    t = torch.randint(0, 10, (4,))
    oa.zero_grad()
    F.nll_loss(a.eval()(x), t).backward()
    oa.step()
    checkpoint.save_checkpoint(a, oa, tmp_path / "model.pth", tmp_path / "optimizer.pth")
    # the files load into stock torch objects
    b = _plain_lenet()
    b.load_state_dict(torch.load(tmp_path / "model.pth", weights_only=True))
    ob = torch.optim.SGD(b.parameters(), lr=0.01, momentum=0.5)
    ob.load_state_dict(torch.load(tmp_path / "optimizer.pth", weights_only=True))
    assert set(ob.state_dict()["state"].keys()) == set(range(8))
    assert ob.state_dict()["param_groups"][0]["momentum"] == 0.5
    # and resume into ours: next step identical to torch's next step
    c = Net()
    oc = FusedSGD(c.parameters(), lr=0.01, momentum=0.5)
    checkpoint.load_checkpoint(c, oc, tmp_path / "model.pth", tmp_path / "optimizer.pth")
    x2 = torch.randn(4, 1, 28, 28)
    for m, o in ((b, ob), (c, oc)):
        m.eval()
        o.zero_grad()
        F.nll_loss(Net.reference_forward(m, x2) if m is b else m.eval()(x2), t).backward()
        o.step()
    for p, q in zip(b.parameters(), c.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-6, atol=1e-7)


def test_flat_params_views_and_grads():
    net = Net()
    fp = FlatParams(list(net.parameters()))
    assert fp.numel == 21840 and fp.data.numel() % 4 == 0
    net.conv1.weight.data.fill_(3.0)
    assert torch.all(fp.data[:250] == 3.0)
    assert fp.grads_are_views()
    net.zero_grad(set_to_none=True)
    F.nll_loss(net.eval()(torch.randn(2, 1, 28, 28)), torch.tensor([1, 2])).backward()
    assert not fp.grads_are_views()
    fp.gather_grads()
    assert fp.grads_are_views() and fp.grad.abs().sum() > 0
