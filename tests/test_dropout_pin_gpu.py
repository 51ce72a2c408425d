"""Dropout inside the fused training kernels, pinned against a reference.

The reference model applies Dropout2d after conv2 and dropout after fc1 in every training step
(ref src/model.py:11,17,20).  The fused kernels draw both masks on the device from Philox4x32-10
(csrc/common.h dropout_keep), keyed by (seed, device step counter, rank * B + batch position,
unit): 20 Dropout2d channels then 50 fc1 units per sample (csrc/kernels/lenet_fused.hip stage 0,
lenet_fused_f32.hip stage 0).  Bit parity with torch's CPU generator is impossible, so:

* the masks are READ BACK from the kernels (with conv2 / fc1 biases large enough that every
  pre-dropout activation is positive, a zero in the per-sample fc vectors the kernel writes is
  exactly a dropped unit) and must equal the host Philox reference bit for bit
  (``ops.rng.philox_uniform_reference``), per (sample, channel) for Dropout2d;
* their statistics: keep rate ~ 1 - p, fresh masks every step, different masks on another rank;
* the split step's four workgroups per sample draw the same masks as one workgroup per sample;
* with the host-regenerated masks applied in the CPU fp32 ``Net``, the exact-fp32 kernel's
  gradients match to 1e-4 relative L2 for every parameter at p = 0.5.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist
from csed_514_project_distributed_training_using_pytorch_amd.data.mnist import MNIST_MEAN, MNIST_STD
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer
from csed_514_project_distributed_training_using_pytorch_amd.models import Net
from csed_514_project_distributed_training_using_pytorch_amd.ops.rng import philox_uniform_reference

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
V_P2, V_H = 0, 384  # per-sample vector slab: fc1 input (after Dropout2d) | fc1 output (after dropout)


def host_masks(seed, counter, rank, B, p):
    """Keep masks of one step as the kernels draw them: [B, 20] Dropout2d channels, [B, 50] units."""
    e = (np.arange(B, dtype=np.uint64)[:, None] + np.uint64(rank * B)) * np.uint64(70) + np.arange(70, dtype=np.uint64)
    u = philox_uniform_reference(seed, counter << 20, e)
    keep = u >= np.float32(p)
    return torch.from_numpy(keep[:, :20].copy()), torch.from_numpy(keep[:, 20:].copy())


def _positive_net():
    """Biases that keep every pre-dropout activation positive: a zero after dropout is a drop."""
    torch.manual_seed(1)
    net = Net()
    with torch.no_grad():
        net.conv2.bias.fill_(8.0)
        net.fc1.weight.mul_(0.01)
        net.fc1.bias.fill_(4.0)
    return net


def _kernel_masks(eng, B):
    """(Dropout2d [B, 20] keep, per-channel all-or-nothing, dropout [B, 50] keep) read back from the
    vector slab the training kernel wrote for the batch at the cursor."""
    eng.gradient()
    torch.cuda.synchronize()
    v = eng.fc_vectors(B).cpu()
    p2 = v[:, V_P2:V_P2 + 320].view(B, 20, 16) != 0
    h = v[:, V_H:V_H + 50] != 0
    return p2.any(2), bool((p2.all(2) == p2.any(2)).all()), h


@pytest.mark.parametrize("dt,B,split", [(torch.bfloat16, 64, True), (torch.bfloat16, 8, True),
                                        (torch.bfloat16, 64, False), (torch.float16, 100, False),
                                        (torch.float32, 64, False), (torch.float32, 100, False),
                                        (torch.float32, 64, True), (torch.float32, 8, True)])
def test_kernel_masks_equal_host_philox(dt, B, split):
    p, seed = 0.5, 1234
    data = synthetic_mnist(256, seed=2)
    eng = FusedLeNetTrainer(_positive_net().to(DEV), data, global_batch=B, compute_dtype=dt, drop_p=p, seed=seed,
                            split=split)
    eng.set_epoch_order(torch.randperm(256, generator=torch.Generator().manual_seed(0))[:B])
    for counter in (0, 3):
        eng.rng_offset.fill_(counter)
        d2, whole, d1 = _kernel_masks(eng, B)
        h2, h1 = host_masks(seed, counter, 0, B, p)
        assert whole, "Dropout2d must drop whole channels (one draw per sample and channel)"
        assert torch.equal(d2, h2)
        assert torch.equal(d1, h1)


def test_mask_statistics_steps_and_ranks():
    """Keep rate ~ 1 - p over 256 samples x 70 units; masks change with the step counter and
    with the rank (same batch, same step); p = 0.25 keeps ~75 %."""
    B = 256
    data = synthetic_mnist(B, seed=2)
    ops = torch.ops.csed
    for p in (0.5, 0.25):
        eng = FusedLeNetTrainer(_positive_net().to(DEV), data, global_batch=B, drop_p=p, seed=99)
        eng.set_epoch_order(torch.arange(B))
        d2, whole, d1 = _kernel_masks(eng, B)
        keep = torch.cat([d2.flatten(), d1.flatten()]).float().mean().item()
        assert whole and abs(keep - (1 - p)) < 0.02, keep
        eng.rng_offset.fill_(1)
        d2b, _, d1b = _kernel_masks(eng, B)
        same_step = torch.cat([(d2 == d2b).flatten(), (d1 == d1b).flatten()]).float().mean().item()
        # rank 1, step 0: the same kernel launched with rank id 1 on the same batch
        eng.rng_offset.fill_(0)
        ops.lenet_train(eng.train_data.images, eng.train_data.labels, eng.perm, eng.cursor, B, 1, eng.wimg,
                        eng.flat.data, eng.slab, eng.vslab, eng.loss_parts, 1.0 / B, MNIST_MEAN, MNIST_STD, p,
                        99, eng.rng_offset, eng.grid, eng.mfma, None, None, None, False)
        torch.cuda.synchronize()
        v = eng.fc_vectors(B).cpu()
        r2 = (v[:, V_P2:V_P2 + 320].view(B, 20, 16) != 0).any(2)
        r1 = v[:, V_H:V_H + 50] != 0
        h2, h1 = host_masks(99, 0, 1, B, p)
        assert torch.equal(r2, h2) and torch.equal(r1, h1)
        cross_rank = torch.cat([(d2 == r2).flatten(), (d1 == r1).flatten()]).float().mean().item()
        agree = p * p + (1 - p) * (1 - p)  # independent draws
        assert abs(same_step - agree) < 0.03, same_step
        assert abs(cross_rank - agree) < 0.03, cross_rank


@pytest.mark.parametrize("B", [64, 8])
def test_split_parts_share_masks(B):
    """With dropout on, the split step (4 workgroups per sample, each running the forward with
    its own draw) computes the one-workgroup-per-sample gradient: identical loss, fc gradients
    bit for bit, conv gradients up to summation order.  A part drawing other masks would put
    another network's conv2 weight-gradient columns into the slab."""
    data = synthetic_mnist(256, seed=23)
    order = torch.randperm(256, generator=torch.Generator().manual_seed(1))[:B]
    res = []
    for split in (True, False):
        torch.manual_seed(3)
        eng = FusedLeNetTrainer(Net().to(DEV), data, global_batch=B, drop_p=0.5, split=split, seed=7)
        assert eng.split == split
        eng.set_epoch_order(order)
        eng.rng_offset.fill_(5)
        g = eng.gradient()
        torch.cuda.synchronize()
        res.append((g.cpu(), eng.loss_acc.clone().cpu()))
    (gs, ls), (g1, l1) = res
    assert torch.equal(ls, l1)
    off = 0
    for name, p in Net().named_parameters():
        n = p.numel()
        a, b = gs[off:off + n], g1[off:off + n]
        if name.startswith("fc"):
            assert torch.equal(a, b), name
        else:
            rel = ((a - b).norm() / b.norm()).item()
            assert rel < 2e-2, (name, rel)
        off += n


def _x(data, idx):
    inv255 = torch.tensor(1.0 / 255.0, dtype=torch.float32)
    inv_std = torch.tensor(1.0, dtype=torch.float32) / torch.tensor(MNIST_STD, dtype=torch.float32)
    x = (data.images[idx].float() * inv255 - torch.tensor(MNIST_MEAN, dtype=torch.float32)) * inv_std
    return x.view(-1, 1, 28, 28)


def _ref_forward_with_masks(net, x, d2, d1, p):
    """ref src/model.py:15-22 with the given Dropout2d / dropout keep masks (train mode)."""
    s = 1.0 / (1.0 - p)
    h = F.relu(F.max_pool2d(net.conv1(x), 2))
    y = net.conv2(h) * (d2.float() * s)[:, :, None, None]
    h = F.relu(F.max_pool2d(y, 2)).view(-1, 320)
    h = F.relu(net.fc1(h)) * (d1.float() * s)
    return F.log_softmax(net.fc2(h), dim=1)


@pytest.mark.parametrize("B,counter", [(64, 0), (100, 7)])
def test_f32_dropout_gradient_matches_cpu_reference(B, counter):
    """Exact-fp32 kernel at p = 0.5 vs the CPU fp32 Net with the same (host-regenerated) masks:
    every parameter's gradient to 1e-4 relative L2, the loss to 1e-5."""
    p, seed = 0.5, 31
    data = synthetic_mnist(256, seed=11)
    torch.manual_seed(1)
    net, ref = Net(), Net()
    ref.load_state_dict(net.state_dict())
    eng = FusedLeNetTrainer(net.to(DEV), data, global_batch=B, compute_dtype=torch.float32, drop_p=p, seed=seed)
    order = torch.randperm(256, generator=torch.Generator().manual_seed(B))[:B]
    eng.set_epoch_order(order)
    eng.rng_offset.fill_(counter)
    g = eng.gradient().cpu()
    d2, d1 = host_masks(seed, counter, 0, B, p)
    out = _ref_forward_with_masks(ref, _x(data, order), d2, d1, p)
    loss = F.nll_loss(out, data.labels[order])
    loss.backward()
    lsum, _ = eng.loss_acc.tolist()
    assert abs(lsum / B - loss.item()) < 1e-5 * max(1.0, loss.item())
    off = 0
    for name, prm in ref.named_parameters():
        n = prm.numel()
        rel = ((g[off:off + n].view_as(prm).double() - prm.grad.double()).norm() / prm.grad.double().norm()).item()
        assert rel < 1e-4, f"{name}: relative L2 error {rel:.3e}"
        off += n
