"""Fused LeNet engine (csrc/kernels/lenet_fused.hip) vs the fp32 PyTorch reference Net."""
import math

import pytest
import torch
import torch.nn.functional as F

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist
from csed_514_project_distributed_training_using_pytorch_amd.data.mnist import MNIST_MEAN, MNIST_STD
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer
from csed_514_project_distributed_training_using_pytorch_amd.models import Net

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _ref_batch(data, idx, dt):
    x = (data.images[idx].float() / 255.0 - MNIST_MEAN) / MNIST_STD
    return x.to(dt).float().view(-1, 1, 28, 28), data.labels[idx]


def _rel(a, b):
    return ((a.float().cpu() - b.float().cpu()).norm() / b.float().cpu().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("dt,tol", [(torch.bfloat16, 6e-2), (torch.float16, 2.5e-2)])
@pytest.mark.parametrize("B,grid", [(64, 64), (64, 16), (8, 8), (100, 7), (64, None), (8, None)])
def test_fused_gradient_matches_reference(dt, tol, B, grid):
    data = synthetic_mnist(256, seed=11)
    torch.manual_seed(1)
    net = Net()
    ref = Net()
    ref.load_state_dict(net.state_dict())
    eng = FusedLeNetTrainer(net.to(DEV), data, lr=0.01, momentum=0.5, global_batch=B, compute_dtype=dt,
                            drop_p=0.0, grid=grid)
    order = torch.randperm(256)[:B]
    eng.set_epoch_order(order)
    g = eng.gradient()
    torch.cuda.synchronize()
    x, t = _ref_batch(data, order, dt)
    ref.eval()  # dropout off, same as drop_p = 0
    out = ref(x)
    loss = F.nll_loss(out, t)
    loss.backward()
    # loss / accuracy partials
    lsum, correct = eng.loss_acc.tolist()
    assert abs(lsum / B - loss.item()) < 3 * tol * max(1.0, loss.item())
    assert abs(correct - (out.argmax(1) == t).sum().item()) <= max(1, B // 20)
    # conv gradients flow through max-pool argmax and ReLU decisions: the fp32
    # reference itself moves by 3-8 % (L2) under a 1e-3 relative input
    # perturbation (see test_reference_sensitivity), so a 16-bit forward can only
    # be held to that band there; the exact check is test_fused_matches_modular.
    off = 0
    for name, p in ref.named_parameters():
        n = p.numel()
        rel = _rel(g[off:off + n].view_as(p), p.grad)
        bound = tol if name.startswith("fc") else CONV_TOL[dt]
        assert rel < bound, f"{name}: relative L2 error {rel:.3e} (bound {bound})"
        off += n


CONV_TOL = {torch.bfloat16: 0.2, torch.float16: 0.08}


def _modular_grads(net, data, order, dt):
    from csed_514_project_distributed_training_using_pytorch_amd import ops
    from csed_514_project_distributed_training_using_pytorch_amd.data import DeviceLoader

    ops.set_compute_dtype(dt)
    try:
        loader = DeviceLoader(data, batch_size=len(order), device=DEV, dtype=dt)
        x, t = loader.batch(order.to(DEV))
        net.eval()
        net.zero_grad(set_to_none=True)
        out = net(x)
        ops.nll_loss(out, t).backward()
        return torch.cat([p.grad.reshape(-1) for p in net.parameters()])
    finally:
        ops.set_compute_dtype(torch.bfloat16)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_fused_matches_modular(dt):
    """Fused kernel vs the per-op HIP path: both make identical pooling/ReLU
    decisions (same MFMA accumulation order per tile), so gradients must agree
    to accumulation-order rounding."""
    data = synthetic_mnist(256, seed=21)
    torch.manual_seed(3)
    net = Net().to(DEV)
    B = 64
    order = torch.randperm(256)[:B]
    eng = FusedLeNetTrainer(net, data, global_batch=B, compute_dtype=dt, drop_p=0.0)
    eng.set_epoch_order(order)
    g = eng.gradient()
    gm = _modular_grads(net, data, order, dt)
    off = 0
    for name, p in net.named_parameters():
        n = p.numel()
        rel = _rel(g[off:off + n], gm[off:off + n])
        assert rel < 2e-2, f"{name}: fused vs modular relative L2 error {rel:.3e}"
        off += n


def test_reference_sensitivity():
    """Documents why conv gradients get a wide band against the fp32 reference."""
    torch.manual_seed(1)
    net = Net().double().eval()
    data = synthetic_mnist(64, seed=11)
    x = ((data.images.double() / 255 - MNIST_MEAN) / MNIST_STD).view(64, 1, 28, 28)
    t = data.labels

    def grads(inp):
        net.zero_grad(set_to_none=True)
        F.nll_loss(net(inp), t).backward()
        return net.conv1.weight.grad.clone()

    g0 = grads(x)
    g1 = grads(x * (1 + 1e-3 * torch.randn_like(x)))
    assert ((g1 - g0).norm() / g0.norm()).item() > 5e-3


def test_fused_sgd_step_and_counters():
    data = synthetic_mnist(128, seed=5)
    torch.manual_seed(1)
    net = Net()
    eng = FusedLeNetTrainer(net.to(DEV), data, lr=0.05, momentum=0.5, global_batch=32, drop_p=0.0)
    p0 = eng.flat.data.clone()
    eng.set_epoch_order(torch.arange(128))
    # gradient of the first batch through the reduce-only path
    g = eng.gradient()
    eng.step()
    torch.cuda.synchronize()
    torch.testing.assert_close(eng.flat.data, p0 - 0.05 * g, rtol=1e-5, atol=1e-6)
    assert eng.step_count.item() == 1 and eng.cursor.item() == 1 and eng.rng_offset.item() == 1
    assert eng.ticket.item() == 0
    # the model's parameters are views of the engine's flat buffer
    torch.testing.assert_close(net.conv1.weight.detach().reshape(-1), eng.flat.data[:250])
    # weight images were refreshed: a re-pack yields identical bytes
    before = eng.wimg.clone()
    eng.repack()
    assert torch.equal(before, eng.wimg)


def test_fused_eval_matches_reference():
    data = synthetic_mnist(1000, seed=9, train=False)
    torch.manual_seed(2)
    net = Net()
    ref = Net()
    ref.load_state_dict(net.state_dict())
    eng = FusedLeNetTrainer(net.to(DEV), synthetic_mnist(64, seed=1), global_batch=64)
    lsum, correct = eng.evaluate(data)
    logp = eng.eval_logp(data)
    x, t = _ref_batch(data, torch.arange(1000), torch.bfloat16)
    ref.eval()
    out = ref(x)
    assert _rel(logp, out) < 2e-2
    ref_sum = F.nll_loss(out, t, reduction="sum").item()
    assert abs(lsum - ref_sum) / ref_sum < 2e-2
    assert abs(correct - (out.argmax(1) == t).sum().item()) <= 10


def test_fused_training_converges_with_dropout_and_graphs():
    """Three epochs over 12,800 samples of the (deliberately hard) synthetic set with dropout
    and graph replay: the test NLL must fall well below chance and accuracy must rise far
    above 10 % (the CPU reference reaches 86 % after a full 60k epoch)."""
    n = 12800
    train = synthetic_mnist(n, seed=3)
    test = synthetic_mnist(1000, seed=4, train=False)
    torch.manual_seed(1)
    net = Net()
    eng = FusedLeNetTrainer(net.to(DEV), train, lr=0.02, momentum=0.5, global_batch=64)
    l0, _ = eng.evaluate(test)
    for epoch in range(3):
        g = torch.Generator()
        g.manual_seed(epoch)
        eng.train_epoch(torch.randperm(n, generator=g), steps_per_graph=8)
    torch.cuda.synchronize()
    l1, c1 = eng.evaluate(test)
    assert math.isfinite(l1)
    assert l1 < 0.5 * l0, (l0, l1)
    assert c1 > 600, c1
    assert eng.capture_comm_ok is True
    assert eng.step_count.item() == 3 * (n // 64)


@pytest.mark.parametrize("B", [64, 24])
def test_batch_staging_is_bitwise_transparent(B):
    """lenet_update gathering the next batch one step ahead (and lenet_train reading it)
    must give exactly the parameters of the perm/cursor path, eager and graph-replayed,
    across an epoch boundary."""
    data = synthetic_mnist(B * 6 + 5, seed=5)
    finals = []
    for staged in (True, False):
        torch.manual_seed(1)
        eng = FusedLeNetTrainer(Net().to(DEV), data, lr=0.05, momentum=0.5, global_batch=B, split=False)
        assert eng.staged
        eng.staged = staged
        g = torch.Generator().manual_seed(7)
        eng.set_epoch_order(torch.randperm(len(data), generator=g))
        eng.run_steps(2, use_graph=False)
        eng.run_steps(3, steps_per_graph=3)
        eng.last_partial_step()
        eng.set_epoch_order(torch.randperm(len(data), generator=g))
        eng.run_steps(4, steps_per_graph=2)
        torch.cuda.synchronize()
        finals.append((eng.flat.data.clone(), eng.loss_acc.clone(), eng.cursor.item()))
    assert torch.equal(finals[0][0], finals[1][0])
    assert torch.equal(finals[0][1], finals[1][1])
    assert finals[0][2] == finals[1][2] == 4


@pytest.mark.parametrize("dtype,band", [(torch.bfloat16, 0.05), (torch.float16, 0.03)])
def test_fused_trajectory_matches_cpu_reference(dtype, band):
    """50 SGD steps with dropout off: the fused GPU engine vs the reference recipe on the CPU
    (stock fp32 ``Net`` + ``torch.optim.SGD``, ref src/train.py:69-85), same initial weights,
    same batches in the same order.  The per-step training losses must track each other
    within the dtype's band over the whole trajectory, and so must the final weights."""
    n, B, steps = 64 * 50, 64, 50
    data = synthetic_mnist(n, seed=17)
    order = torch.randperm(n, generator=torch.Generator().manual_seed(3))
    torch.manual_seed(1)
    ref = Net()
    net = Net()
    net.load_state_dict(ref.state_dict())
    eng = FusedLeNetTrainer(net.to(DEV), data, lr=0.02, momentum=0.5, global_batch=B, compute_dtype=dtype,
                            drop_p=0.0)
    eng.set_epoch_order(order)
    opt = torch.optim.SGD(ref.parameters(), lr=0.02, momentum=0.5)
    ref.eval()  # no dropout (Net has no other train/eval difference)
    x_all = ((data.images.float() / 255.0 - MNIST_MEAN) / MNIST_STD).unsqueeze(1)
    gpu_l, cpu_l = [], []
    for s in range(steps):
        eng.step()
        lsum, _ = eng.take_loss()
        gpu_l.append(lsum / B)
        idx = order[s * B:(s + 1) * B]
        opt.zero_grad()
        loss = F.nll_loss(ref(x_all[idx]), data.labels[idx])
        loss.backward()
        opt.step()
        cpu_l.append(loss.item())
    gl, cl = torch.tensor(gpu_l), torch.tensor(cpu_l)
    assert cl[-10:].mean() < 0.9 * cl[:5].mean()  # the reference itself learned something
    assert ((gl - cl).abs() / cl).max() < band, list(zip(gpu_l, cpu_l))
    for (name, p_ref), p in zip(ref.named_parameters(), net.parameters()):
        assert _rel(p.detach().cpu(), p_ref.detach()) < band, name


@pytest.mark.parametrize("B", [64, 8, 24])
def test_split_step_matches_one_workgroup_per_sample(B):
    """The split step (4 workgroups per sample dividing the backward conv stages) computes the
    same gradient as one workgroup per sample, up to summation order (dgrad K parts, conv1
    wgrad partials summed by lenet_update); loss and accuracy are identical."""
    data = synthetic_mnist(256, seed=23)
    order = torch.randperm(256, generator=torch.Generator().manual_seed(1))[:B]
    res = []
    for split in (True, False):
        torch.manual_seed(3)
        eng = FusedLeNetTrainer(Net().to(DEV), data, global_batch=B, drop_p=0.0, split=split)
        assert eng.split == split and eng.grid == (4 * B if split else B)
        eng.set_epoch_order(order)
        g = eng.gradient()
        torch.cuda.synchronize()
        res.append((g, eng.loss_acc.clone()))
    (gs, ls), (g1, l1) = res
    assert torch.equal(ls, l1)
    net = Net()
    off = 0
    for name, p in net.named_parameters():
        n = p.numel()
        rel = _rel(gs[off:off + n], g1[off:off + n])
        assert rel < 2e-2, f"{name}: split vs one-workgroup relative L2 error {rel:.3e}"
        if name.startswith("fc"):
            assert torch.equal(gs[off:off + n], g1[off:off + n]), name  # fc grads: same kernel path
        off += n


def test_split_step_trains_and_replays_bitwise():
    """Graph-replayed split steps across an epoch boundary (with the tail step) equal the same
    steps launched eagerly, bit for bit; staging rows stay per workgroup."""
    data = synthetic_mnist(64 * 5 + 17, seed=5)
    finals = []
    for use_graph in (True, False):
        torch.manual_seed(1)
        eng = FusedLeNetTrainer(Net().to(DEV), data, lr=0.05, momentum=0.5, global_batch=64)
        assert eng.split and eng.grid == 256 and eng.xstage.shape[0] == 256
        g = torch.Generator().manual_seed(7)
        for _ in range(2):
            eng.train_epoch(torch.randperm(len(data), generator=g), steps_per_graph=2, use_graph=use_graph)
        torch.cuda.synchronize()
        finals.append((eng.flat.data.clone(), eng.loss_acc.clone()))
    assert torch.equal(finals[0][0], finals[1][0]) and torch.equal(finals[0][1], finals[1][1])
    assert torch.isfinite(finals[0][0]).all()


@pytest.mark.parametrize("B", [64, 8])
def test_native_stepper_matches_graphs_and_eager(B):
    """The native step executor (csed.LenetStepper: argument blocks built once, 2k launches
    from C++) runs exactly the steps that graph replay and per-step Python launches run,
    across an epoch boundary and a tail step, bit for bit; it is rebuilt when the epoch
    buffer changes."""
    data = synthetic_mnist(B * 7 + 3, seed=9)
    finals = []
    for mode in ("native", "graph", "python"):
        torch.manual_seed(1)
        eng = FusedLeNetTrainer(Net().to(DEV), data, lr=0.05, momentum=0.5, global_batch=B)
        eng.native_max = 64 if mode == "native" else 0
        g = torch.Generator().manual_seed(7)
        for _ in range(2):
            eng.set_epoch_order(torch.randperm(len(data), generator=g))
            if mode == "python":
                for _ in range(eng.full_steps()):
                    eng.step()
            else:
                plan = eng.step_plan(3, 2)
                assert len(plan) == 1 if mode == "native" else len(plan) == 2
                for launch in plan:
                    launch()
                eng.run_steps(eng.full_steps() - 3, 2, use_graph=mode == "graph")
            eng.last_partial_step(use_graph=mode == "graph")
        torch.cuda.synchronize()
        finals.append((eng.flat.data.clone(), eng.momentum_buf.clone(), eng.loss_acc.clone(),
                       eng.step_count.item()))
    for other in finals[1:]:
        assert torch.equal(finals[0][0], other[0]) and torch.equal(finals[0][1], other[1])
        assert torch.equal(finals[0][2], other[2]) and finals[0][3] == other[3] == 2 * 8
