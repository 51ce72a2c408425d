"""The per-op kernel library in exact fp32 (``ops.set_compute_dtype(torch.float32)``: fp32
operands in LDS, each 16x16x32 K-slice as eight v_mfma_f32_16x16x4_f32, common.h Mfma<float>)
against the plain PyTorch fp32 ops: agreement to fp32 summation-order rounding (~1e-6),
orders of magnitude inside the 16-bit bands of test_kernels_gpu.py."""
import pytest
import torch
import torch.nn.functional as F

from csed_514_project_distributed_training_using_pytorch_amd import ops
from csed_514_project_distributed_training_using_pytorch_amd.ops import _native

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _fp32():
    _native.require()
    ops.set_compute_dtype(torch.float32)
    yield
    ops.set_compute_dtype(torch.bfloat16)


def close(a, b, rel=2e-5, name=""):
    a = a.float().cpu()
    b = b.float().cpu()
    scale = max(b.abs().max().item(), 1e-6)
    err = (a - b).abs().max().item()
    assert err <= rel * scale, f"{name}: max err {err:.3e} vs scale {scale:.3e}"


@pytest.mark.parametrize("shape", [(4, 1, 28, 28, 10, 5, 0), (3, 10, 12, 12, 20, 5, 0), (2, 3, 9, 11, 7, 3, 1),
                                   (2, 16, 14, 14, 33, 3, 1)])
def test_conv2d_fwd_bwd_fp32(shape):
    N, C, H, W, OC, K, pad = shape
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W)
    w = torch.randn(OC, C, K, K) * 0.2
    b = torch.randn(OC)
    xg = x.to(DEV).requires_grad_(True)
    wg = w.to(DEV).requires_grad_(True)
    bg = b.to(DEV).requires_grad_(True)
    y = ops.conv2d(xg, wg, bg, padding=pad)
    assert y.dtype == torch.float32
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    yr = F.conv2d(xr, wr, br, padding=pad)
    close(y, yr, name="conv fwd")
    gy = torch.randn(yr.shape)
    y.backward(gy.to(DEV))
    yr.backward(gy)
    close(xg.grad, xr.grad, name="conv dgrad")
    close(wg.grad, wr.grad, name="conv wgrad")
    close(bg.grad, br.grad, name="conv bgrad")


@pytest.mark.parametrize("mnk", [(64, 50, 320), (8, 10, 50), (37, 70, 45), (4096, 50, 320)])
def test_linear_fp32(mnk):
    M, N, K = mnk
    torch.manual_seed(3)
    x, w, b = torch.randn(M, K), torch.randn(N, K) * 0.1, torch.randn(N)
    xg = x.to(DEV).requires_grad_(True)
    wg, bg = w.to(DEV).requires_grad_(True), b.to(DEV).requires_grad_(True)
    y = ops.linear(xg, wg, bg, act="relu", out_dtype=torch.float32)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    yr = F.relu(F.linear(xr, wr, br))
    close(y, yr, name="linear fwd")
    gy = torch.randn(yr.shape)
    y.backward(gy.to(DEV))
    yr.backward(gy)
    close(xg.grad, xr.grad, name="linear dx")
    close(wg.grad, wr.grad, name="linear dw")
    close(bg.grad, br.grad, name="linear db")


def test_net_fp32_matches_reference_forward_backward():
    """The whole Net through the op library in fp32: every gradient, conv included, within
    1e-4 relative L2 of the CPU reference (the 16-bit path is held to 20 % on conv)."""
    from csed_514_project_distributed_training_using_pytorch_amd.models import Net

    torch.manual_seed(1)
    net = Net().eval()
    ref = Net().eval()
    ref.load_state_dict(net.state_dict())
    net = net.to(DEV)
    x = torch.randn(64, 1, 28, 28)
    t = torch.randint(0, 10, (64,))
    out = net(x.to(DEV))
    loss = ops.nll_loss(out, t.to(DEV))
    loss.backward()
    out_r = ref(x)
    F.nll_loss(out_r, t).backward()
    close(out, out_r, rel=1e-5, name="net logp")
    for (n1, p1), (_, p2) in zip(net.named_parameters(), ref.named_parameters()):
        a, b = p1.grad.float().cpu(), p2.grad
        rel = ((a - b).norm() / b.norm()).item()
        assert rel < 1e-4, f"grad {n1}: relative L2 error {rel:.3e}"


def test_fused_fp32_matches_modular_fp32():
    """The two fp32 implementations (fused lenet_train_f32 and the per-op library) agree on
    one batch's gradient to fp32 rounding."""
    from csed_514_project_distributed_training_using_pytorch_amd.data import DeviceLoader, synthetic_mnist
    from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer
    from csed_514_project_distributed_training_using_pytorch_amd.models import Net

    data = synthetic_mnist(256, seed=21)
    torch.manual_seed(3)
    net = Net().to(DEV)
    order = torch.randperm(256)[:64]
    eng = FusedLeNetTrainer(net, data, global_batch=64, compute_dtype=torch.float32, drop_p=0.0)
    eng.set_epoch_order(order)
    g = eng.gradient()
    loader = DeviceLoader(data, batch_size=64, device=DEV, dtype=torch.float32)
    x, t = loader.batch(order.to(DEV))
    net.eval()
    net.zero_grad(set_to_none=True)
    ops.nll_loss(net(x), t).backward()
    gm = torch.cat([p.grad.reshape(-1) for p in net.parameters()])
    off = 0
    for name, p in net.named_parameters():
        n = p.numel()
        rel = ((g[off:off + n] - gm[off:off + n]).norm() / gm[off:off + n].norm()).item()
        assert rel < 1e-4, f"{name}: fused vs modular fp32 relative L2 error {rel:.3e}"
        off += n
