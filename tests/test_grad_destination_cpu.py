"""Gradient destinations of the modular engine (ops/functional.py set_grad_destination): a
registered parameter whose .grad is None gets its gradient written into the registered buffer
(a fresh view each time, so autograd adopts it without a copy); one that already holds a gradient
gets a fresh buffer, so accumulation keeps torch's semantics.  CPU: the selection logic and
autograd's adoption are device-independent."""
import torch

from csed_514_project_distributed_training_using_pytorch_amd.ops import functional as F
from csed_514_project_distributed_training_using_pytorch_amd.ops.rng import PhiloxState


class _Scale(torch.autograd.Function):
    """y = x * w with dL/dw written through F._grad_buffer (as the conv / linear backward do)."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x)
        ctx.w = w
        return x * w

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        dw = F._grad_buffer(ctx.w, ctx.w.shape, ctx.w.device)
        dw.copy_((g * x).sum(0))
        return None, dw


def test_backward_writes_into_registered_buffer_and_accumulates():
    w = torch.nn.Parameter(torch.ones(4))
    flat = torch.zeros(6)
    F.set_grad_destination(w, flat[1:5])
    x = torch.arange(8.0).view(2, 4)
    _Scale.apply(x, w).sum().backward()
    assert w.grad.data_ptr() == flat[1:5].data_ptr()  # adopted, not copied
    torch.testing.assert_close(flat[1:5], x.sum(0))
    # a second backward without zero_grad accumulates (fresh buffer, then AccumulateGrad's add)
    _Scale.apply(x, w).sum().backward()
    torch.testing.assert_close(flat[1:5], 2 * x.sum(0))
    # set_to_none, then the next backward writes in place again
    w.grad = None
    _Scale.apply(2 * x, w).sum().backward()
    torch.testing.assert_close(flat[1:5], 2 * x.sum(0))
    assert w.grad.data_ptr() == flat[1:5].data_ptr()
    F.set_grad_destination(w, None)
    w.grad = None
    _Scale.apply(x, w).sum().backward()
    assert w.grad.data_ptr() != flat[1:5].data_ptr()


def test_destination_shape_is_checked():
    w = torch.nn.Parameter(torch.ones(3))
    try:
        F.set_grad_destination(w, torch.zeros(4))
    except ValueError:
        return
    raise AssertionError("a destination of the wrong shape must be rejected")


def test_philox_offsets_restart_per_step():
    st = PhiloxState(seed=7)
    a = [st.next()[1] for _ in range(3)]
    st.reset_offset()
    b = [st.next()[1] for _ in range(3)]
    assert a == b == [0, 1, 2]
