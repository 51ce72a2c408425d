"""Differentiable ops backed by the gfx950 HIP kernels (``torch.ops.csed``).

Device dispatch is by tensor device only: GPU tensors always go through the
hand-written kernels (and raise if the extension is missing); CPU tensors use
the stock PyTorch ops, which serve as the fp32 numerical oracle for the tests
(SURVEY.md section 4, item 1).

Compute precision on the GPU: activations are stored in the compute dtype
(bf16 by default, fp16 optional), matrix-shaped work runs on
``v_mfma_f32_16x16x32_{bf16,f16}`` with fp32 accumulation, weights stay fp32
masters (the kernels convert while staging them into LDS), and weight
gradients are produced in fp32.  ``set_compute_dtype(torch.float32)`` is the
reference's precision: fp32 activations and operands, each 16x16x32 K-slice
as eight exact ``v_mfma_f32_16x16x4_f32`` (common.h ``Mfma<float>``).

Reference parity map (ref = /root/reference):
  conv2d / conv2d_pool_relu   <- nn.Conv2d, F.max_pool2d, F.relu      src/model.py:9-10,16-17
  dropout / dropout2d         <- F.dropout, nn.Dropout2d              src/model.py:11,17,20
  linear                      <- nn.Linear (+relu, +dropout fused)    src/model.py:12-13,19-21
  log_softmax, nll_loss       <- F.log_softmax, F.nll_loss             src/model.py:22, src/train.py:74
  cross_entropy               <- nn.CrossEntropyLoss on log-probs      src/train_dist.py:67,82
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _native
from .rng import default_state

_compute_dtype = torch.bfloat16


def set_compute_dtype(dtype: torch.dtype) -> None:
    global _compute_dtype
    if dtype not in (torch.bfloat16, torch.float16, torch.float32):
        raise ValueError("compute dtype must be torch.bfloat16, torch.float16 or torch.float32")
    _compute_dtype = dtype


def compute_dtype() -> torch.dtype:
    return _compute_dtype


def _mfma() -> int:
    return _native.MFMA_CODE[_compute_dtype]


def _ops():
    return _native.ops()


def _act_dtype(x: torch.Tensor) -> torch.dtype:
    """Activation storage dtype: the compute dtype (fp32 activations on the exact-fp32 path)."""
    if _compute_dtype == torch.float32:
        return torch.float32
    return x.dtype if x.dtype in (torch.bfloat16, torch.float16) else _compute_dtype


# Weight-gradient destinations (engine/modular.py): a parameter registered here whose ``.grad``
# is None when its backward runs gets its gradient written straight into the registered buffer
# (a view of the flat gradient), which autograd's AccumulateGrad then adopts as ``.grad`` without
# a copy or an add kernel.  A parameter that already holds a gradient gets a fresh buffer, so
# accumulation (no zero_grad between two backwards) keeps its usual semantics.
#
# A parameter used more than once in one forward (shared weights, a layer applied twice) has one
# backward call per use within ONE autograd pass, and autograd sums their outputs before
# AccumulateGrad.  Only the pass's first call may get the registered buffer (else every call would
# write the same memory and the sum would add aliases of it); the first hand-out is marked, later
# calls of the pass get fresh buffers, and the mark is dropped by a callback queued on the autograd
# engine for the end of the pass (or by the next zero_grad's set_to_none).
import threading  # noqa: E402
import weakref  # noqa: E402

# id(param) -> (weak reference to param, buffer); keyed by identity (tensors compare elementwise)
_grad_dest: dict[int, tuple[weakref.ref, torch.Tensor]] = {}
_handed_out: set[int] = set()  # ids of parameters handed a gradient buffer in the running pass
_lock = threading.Lock()  # (autograd runs one worker thread per device)


def set_grad_destination(param: torch.Tensor, buf: torch.Tensor | None) -> None:
    """Register (or with None, drop) the fp32 buffer ``param``'s gradient is written into."""
    if buf is None:
        _grad_dest.pop(id(param), None)
        return
    if buf.shape != param.shape or buf.dtype != torch.float32 or buf.device != param.device:
        raise ValueError("gradient destination must be an fp32 tensor of the parameter's shape and device")
    for k in [k for k, (r, _) in _grad_dest.items() if r() is None]:  # (drop dead entries)
        del _grad_dest[k]
    _grad_dest[id(param)] = (weakref.ref(param), buf)


def _queue_end_of_pass(fn) -> bool:
    """Run ``fn`` when the running autograd pass ends.  False outside a backward pass."""
    try:
        torch.autograd.Variable._execution_engine.queue_callback(fn)
        return True
    except RuntimeError:
        return False


def _take_grad_buffer(param: torch.Tensor | None, shape, device) -> tuple[torch.Tensor, bool]:
    """(gradient buffer for ``param``, adopted).  Adopted: the buffer is the registered destination,
    the only gradient this pass produces for ``param``, and autograd's AccumulateGrad will take it
    as ``.grad`` as it is -- ``.grad`` is None, grad mode is off (no create_graph) and no earlier
    call of this pass was handed one -- so nothing reads it before the pass's end-of-pass callbacks
    have run (the condition for deferring the conv weight-gradient reduce).  Parameters without a
    registered destination (e.g. under torch's own DDP, whose C++ grad hooks are invisible here)
    never count as adopted."""
    if param is None:
        return torch.empty(shape, device=device, dtype=torch.float32), False
    key = id(param)
    hit = _grad_dest.get(key)
    if hit is None or hit[0]() is not param:
        return torch.empty(shape, device=device, dtype=torch.float32), False
    with _lock:
        first = param.grad is None and key not in _handed_out and not torch.is_grad_enabled()
        if first and _queue_end_of_pass(lambda: _release(key)):
            _handed_out.add(key)
        else:
            first = False
    if first:
        return hit[1].view(hit[1].shape), True  # (a fresh view: AccumulateGrad steals only a sole reference)
    return torch.empty(shape, device=device, dtype=torch.float32), False


def _release(key: int) -> None:
    with _lock:
        _handed_out.discard(key)


def _grad_buffer(param: torch.Tensor | None, shape, device) -> torch.Tensor:
    return _take_grad_buffer(param, shape, device)[0]


def release_grad_buffers(params) -> None:
    """Forget this pass's hand-out marks of ``params`` (zero_grad with set_to_none; a pass that
    raised before its end-of-pass callbacks ran)."""
    with _lock:
        for p in params:
            _handed_out.discard(id(p))


def wgrad_workspace_elems(N: int, IC: int, KH: int, KW: int, OC: int) -> int:
    """Floats of a conv weight-gradient workspace: one [OC, IC*KH*KW + 1] partial slab per block,
    sized for the most blocks csrc/kernels/conv.hip conv2d_wgrad_blocks makes (256, 512 from
    N = 2048; the extension checks the size)."""
    return max(1, min(N, 512 if N >= 2048 else 256)) * OC * (IC * KH * KW + 1)


# The deferred weight-gradient slab reduce.  A conv backward normally ends with its own reduce
# launch (the partial slabs -> dW, db); when deferral is on, no hook watches the parameters (a DDP
# reducer's post-accumulate-grad hooks would read dW before it is final) and autograd will adopt
# dW / db as they are (``_take_grad_buffer``: ``.grad`` None, first use in the pass, no
# create_graph -- an accumulating ``grad += dW`` or a shared weight's sum would be enqueued as soon
# as this backward returns, before the reduce), the reduce is left pending: the NEXT conv backward
# of the same autograd pass on that device runs it as extra blocks of its own launch (it does not
# depend on it), and a callback queued on the autograd engine flushes whatever is still pending
# when the pass ends -- before any optimizer or user code can read the gradients.  One launch
# fewer per step in the modular engine (conv2's reduce rides on conv1's backward).
_defer_reduce = os.environ.get("CSED_DEFER_WGRAD_REDUCE", "1") != "0"
# device index -> (ws, dw, db, N, IC, KH, KW) of the conv whose reduce is pending on that device
# (autograd's per-device worker threads each touch their own entry; the swaps hold _lock)
_pending: dict[int, tuple] = {}


def set_defer_wgrad_reduce(on: bool) -> None:
    """Enable / disable carrying a conv's weight-gradient reduce into the next conv backward."""
    global _defer_reduce
    _defer_reduce = bool(on)


def pending_reduce_count() -> int:
    """Number of weight-gradient reduces still pending (0 after every completed backward)."""
    with _lock:
        return len(_pending)


def _flush_pending_reduce(dev: int | None = None) -> None:
    """Run the pending reduce of device ``dev`` (None: of every device)."""
    with _lock:
        keys = list(_pending) if dev is None else [dev]
        todo = [_pending.pop(k) for k in keys if k in _pending]
    for ws, dw, db, N, IC, KH, KW in todo:
        with torch.cuda.device(dw.device):
            _ops().wgrad_reduce(ws, dw, db, N, IC, KH, KW)


def _watched(t) -> bool:
    return t is not None and bool(getattr(t, "_post_accumulate_grad_hooks", None) or getattr(t, "_backward_hooks", None))


def _unpool_min_batch(with_dx: bool) -> int:
    """Smallest batch whose pooled conv backward materialises dL/dconv first (CSED_UNPOOL_MIN_BATCH
    / CSED_UNPOOL_MIN_BATCH_WGRAD; the fused expansion stays below: one launch fewer)."""
    v = os.environ.get("CSED_UNPOOL_MIN_BATCH" if with_dx else "CSED_UNPOOL_MIN_BATCH_WGRAD")
    return int(v) if v else (1024 if with_dx else 1 << 30)


# ----------------------------------------------------------------- conv ----
# The weight-gradient kernel holds at most 64 output channels (4 M-tiles of accumulators per wave,
# csrc/kernels/conv.hip launch_conv2d_bwd); a wider conv's backward runs per 64-channel slice.
_WGRAD_MAX_OC = 64


def _conv_bwd_oc_chunks(ctx, x, w, dy, pooled):
    """Backward of a conv with more than 64 output channels: dW / db per 64-channel slice of dy and
    W, dX as the sum of the slices' data gradients (fp32).  dL/dconv of a pooled forward is
    materialised first."""
    if pooled[0] is not None:
        idx, y, chscale = pooled
        dconv = torch.empty(ctx.conv_shape, device=dy.device, dtype=y.dtype)
        _ops().maxpool_relu_bwd(dy, y, idx, chscale, dconv, 2)
        dy = dconv
    N, IC = x.shape[:2]
    OC, _, KH, KW = w.shape
    dw = _take_grad_buffer(w, w.shape, w.device)[0] if ctx.needs_input_grad[1] else None
    db = _take_grad_buffer(ctx.bias_param, (OC,), w.device)[0] if ctx.has_bias and ctx.needs_input_grad[2] else None
    dx32 = torch.zeros(x.shape, device=x.device, dtype=torch.float32) if ctx.needs_input_grad[0] else None
    for c0 in range(0, OC, _WGRAD_MAX_OC):
        c1 = min(OC, c0 + _WGRAD_MAX_OC)
        dyc, wc = dy[:, c0:c1].contiguous(), w[c0:c1].contiguous()
        dwc = torch.empty(wc.shape, device=w.device, dtype=torch.float32)
        dbc = torch.empty(c1 - c0, device=w.device, dtype=torch.float32) if ctx.has_bias else None
        ws = torch.empty(wgrad_workspace_elems(N, IC, KH, KW, c1 - c0), device=w.device, dtype=torch.float32)
        dxc = torch.empty(x.shape, device=x.device, dtype=x.dtype) if dx32 is not None else None
        _ops().conv2d_bwd(x, dyc, wc, dwc, dbc, ws, dxc, ctx.pad, None, None, None, ctx.mf)
        if dw is not None:
            dw[c0:c1].copy_(dwc)
        if db is not None:
            db[c0:c1].copy_(dbc)
        if dxc is not None:
            dx32 += dxc.float()
    dx = dx32.to(x.dtype) if dx32 is not None else None
    return dx, dw, db, None, None, None, None


class _Conv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, pad, pool, chscale, drop):
        if _pending:  # (left by a backward pass that did not finish: run it now)
            _flush_pending_reduce()
        x = x.contiguous()
        if x.dtype not in (torch.float32, _compute_dtype):  # (the kernels take fp32 or the compute dtype)
            x = x.to(_compute_dtype)
        N, IC, H, W = x.shape
        OC, _, KH, KW = w.shape
        OH, OW = H + 2 * pad - KH + 1, W + 2 * pad - KW + 1
        adt = _act_dtype(x)
        mf = _mfma()
        if pool:
            y = torch.empty((N, OC, OH // 2, OW // 2), device=x.device, dtype=adt)
            idx = torch.empty(y.shape, device=x.device, dtype=torch.uint8)
            if drop is not None:  # Dropout2d drawn in the conv's epilogue; its scales kept for the backward
                p, seed, off, dev = drop
                chscale = torch.empty(N * OC, device=x.device, dtype=torch.float32)
                _ops().conv2d_fwd(x, w, b, y, pad, idx, None, 2, mf, p, seed, off, dev, chscale)
            else:
                _ops().conv2d_fwd(x, w, b, y, pad, idx, chscale, 2, mf)
            ctx.save_for_backward(x, w, y, idx, chscale)
        else:
            y = torch.empty((N, OC, OH, OW), device=x.device, dtype=adt)
            _ops().conv2d_fwd(x, w, b, y, pad, None, None, 0, mf)
            ctx.save_for_backward(x, w)
        ctx.pad, ctx.pool, ctx.mf, ctx.has_bias = pad, pool, mf, b is not None
        ctx.bias_param = b
        ctx.conv_shape = (N, OC, OH, OW)
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        if ctx.pool:
            x, w, y, idx, chscale = ctx.saved_tensors
            if dy.dtype != y.dtype:
                dy = dy.to(y.dtype)
            pooled = (idx, y, chscale)
            if x.shape[0] >= _unpool_min_batch(ctx.needs_input_grad[0]):
                # large batch: dL/dconv materialised once (one elementwise launch) instead of every
                # weight- / data-gradient block expanding the pooled gradient on load -- 4 loads
                # (value, argmax, gate, scale) per patch element, in dependent rounds
                dconv = torch.empty(ctx.conv_shape, device=dy.device, dtype=y.dtype)
                _ops().maxpool_relu_bwd(dy, y, idx, chscale, dconv, 2)
                dy, pooled = dconv, (None, None, None)
        else:
            x, w = ctx.saved_tensors
            pooled = (None, None, None)
        dx = dw = db = None
        if (ctx.needs_input_grad[1] or ctx.needs_input_grad[2]) and ctx.conv_shape[1] > _WGRAD_MAX_OC:
            return _conv_bwd_oc_chunks(ctx, x, w, dy, pooled)
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            # one launch for dW, db and dX (+ the slab reduce); a pooled forward's gradient is
            # expanded inside the kernels' staging (dL/dconv never materialised)
            N, IC = x.shape[:2]
            OC, _, KH, KW = w.shape
            dw, dw_adopt = _take_grad_buffer(w, w.shape, w.device)
            db, db_adopt = _take_grad_buffer(ctx.bias_param, (OC,), w.device) if ctx.has_bias else (None, True)
            ws = torch.empty(wgrad_workspace_elems(N, IC, KH, KW, OC), device=w.device, dtype=torch.float32)
            if ctx.needs_input_grad[0]:
                dx = torch.empty(x.shape, device=x.device, dtype=x.dtype)
            dev = w.device.index if w.device.index is not None else torch.cuda.current_device()
            with _lock:  # (another conv's reduce on this device rides on this launch)
                carry = _pending.pop(dev, None)
            defer = (_defer_reduce and dw_adopt and db_adopt and ctx.needs_input_grad[1]
                     and (not ctx.has_bias or ctx.needs_input_grad[2])
                     and not _watched(w) and not _watched(ctx.bias_param))
            ck = {} if carry is None else dict(carry_ws=carry[0], carry_dw=carry[1], carry_db=carry[2],
                                               carry_n=carry[3], carry_ic=carry[4], carry_kh=carry[5],
                                               carry_kw=carry[6])
            _ops().conv2d_bwd(x, dy, w, dw, db, ws, dx, ctx.pad, *pooled, ctx.mf, defer_reduce=defer, **ck)
            if defer and _queue_end_of_pass(lambda: _flush_pending_reduce(dev)):
                # (detached aliases: a second reference to dw / db themselves would make autograd's
                # AccumulateGrad clone them -- before the deferred reduce has written them -- not adopt them)
                with _lock:
                    _pending[dev] = (ws, dw.detach(), db.detach() if db is not None else None, N, IC, KH, KW)
            elif defer:  # (not inside an autograd pass: nothing would flush it)
                _ops().wgrad_reduce(ws, dw, db, N, IC, KH, KW)
        elif ctx.needs_input_grad[0]:
            if ctx.pool:
                dconv = torch.empty(ctx.conv_shape, device=dy.device, dtype=y.dtype)
                _ops().maxpool_relu_bwd(dy, y, idx, chscale, dconv, 2)
            else:
                dconv = dy
            dx = torch.empty(x.shape, device=x.device, dtype=x.dtype)
            _ops().conv2d_dgrad(dconv, w, dx, ctx.pad, ctx.mf)
        return dx, dw, db, None, None, None, None


def conv2d(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None, padding: int = 0):
    """nn.functional.conv2d (stride 1, symmetric padding) on MFMA implicit GEMM."""
    if not x.is_cuda:
        return F.conv2d(x, weight, bias, padding=padding)
    return _Conv2d.apply(x, weight, bias, int(padding), False, None, None)


def conv2d_pool_relu(x, weight, bias=None, chscale: torch.Tensor | None = None, padding: int = 0,
                     dropout2d_p: float = 0.0):
    """relu(max_pool2d(dropout2d(conv2d(x)), 2)) in one kernel (ref src/model.py:16-17).

    ``chscale`` is an optional fp32 [N*C] per-channel scale (a Dropout2d mask already divided by
    1-p); ``dropout2d_p > 0`` instead draws the Dropout2d mask inside the kernel (the same Philox
    draw as :func:`dropout2d_scale`, one ``default_state`` offset).
    """
    if not x.is_cuda:
        y = F.conv2d(x, weight, bias, padding=padding)
        if chscale is not None:
            y = y * chscale.view(y.shape[0], y.shape[1], 1, 1).to(y.dtype)
        elif dropout2d_p > 0.0:
            y = F.dropout2d(y, dropout2d_p, True)
        return F.relu(F.max_pool2d(y, 2))
    drop = None
    if chscale is None and dropout2d_p > 0.0:
        seed, off, dev = default_state.next()
        drop = (float(dropout2d_p), seed, off, dev)
    return _Conv2d.apply(x, weight, bias, int(padding), True, chscale, drop)


# ----------------------------------------------------------------- pool ----
class _MaxPoolRelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, chscale):
        x = x.contiguous()
        N, C, H, W = x.shape
        y = torch.empty((N, C, H // k, W // k), device=x.device, dtype=x.dtype)
        idx = torch.empty(y.shape, device=x.device, dtype=torch.uint8)
        _ops().maxpool_relu_fwd(x, y, idx, chscale, k)
        ctx.save_for_backward(y, idx, chscale)
        ctx.k, ctx.xshape = k, x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        y, idx, chscale = ctx.saved_tensors
        dx = torch.empty(ctx.xshape, device=dy.device, dtype=y.dtype)
        _ops().maxpool_relu_bwd(dy.contiguous().to(y.dtype), y, idx, chscale, dx, ctx.k)
        return dx, None, None


def max_pool2d_relu(x, k: int = 2, chscale: torch.Tensor | None = None):
    """relu(max_pool2d(x * chscale, k)) with kernel == stride == k."""
    if not x.is_cuda:
        if chscale is not None:
            x = x * chscale.view(x.shape[0], x.shape[1], 1, 1).to(x.dtype)
        return F.relu(F.max_pool2d(x, k))
    return _MaxPoolRelu.apply(x, int(k), chscale)


# -------------------------------------------------------------- dropout ----
class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, inner, seed, offset, offset_dev):
        x = x.contiguous()
        y = torch.empty_like(x)
        _ops().dropout_fwd(x, y, inner, p, seed, offset, offset_dev)
        ctx.args = (p, inner, seed, offset)
        ctx.save_for_backward(offset_dev) if offset_dev is not None else None
        ctx.has_dev = offset_dev is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        p, inner, seed, offset = ctx.args
        offset_dev = ctx.saved_tensors[0] if ctx.has_dev else None
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        # the mask is a pure function of (seed, offset, element): regenerate it
        _ops().dropout_fwd(dy, dx, inner, p, seed, offset, offset_dev)
        return dx, None, None, None, None, None


def dropout(x, p: float = 0.5, training: bool = True):
    if not training or p == 0.0:
        return x
    if not x.is_cuda:
        return F.dropout(x, p, training)
    seed, off, dev = default_state.next()
    return _Dropout.apply(x, float(p), 0, seed, off, dev)


def dropout2d(x, p: float = 0.5, training: bool = True):
    if not training or p == 0.0:
        return x
    if not x.is_cuda:
        return F.dropout2d(x, p, training)
    seed, off, dev = default_state.next()
    inner = x.shape[2] * x.shape[3]
    return _Dropout.apply(x, float(p), int(inner), seed, off, dev)


def dropout2d_scale(n: int, c: int, p: float, device) -> torch.Tensor:
    """Per-(sample, channel) Dropout2d scale vector (0 or 1/(1-p)), fp32 [n*c]."""
    s = torch.empty(n * c, device=device, dtype=torch.float32)
    if torch.device(device).type != "cuda":
        return (torch.rand(n * c) >= p).float().div_(1.0 - p) if p < 1 else torch.zeros(n * c)
    seed, off, dev = default_state.next()
    _ops().channel_mask(s, float(p), seed, off, dev)
    return s


# --------------------------------------------------------------- linear ----
_ACT = {"none": 0, "relu": 1, "relu_dropout": 2}


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act, p, seed, offset, offset_dev, out_dtype):
        lead = x.shape[:-1]
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        if x2.dtype not in (torch.bfloat16, torch.float16, torch.float32):
            x2 = x2.float()
        y = torch.empty((x2.shape[0], w.shape[0]), device=x.device, dtype=out_dtype)
        _ops().gemm(x2, w.t(), y, b, 1.0, 0.0, act, p, seed, offset, offset_dev, None, 1.0, _mfma())
        ctx.save_for_backward(x2, w, y if act else None)
        ctx.act, ctx.p, ctx.has_bias, ctx.lead = act, p, b is not None, lead
        ctx.bias_param = b
        return y.view(*lead, w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w, y = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0]).contiguous()
        gate = y if ctx.act else None
        if gate is not None and dy2.dtype != gate.dtype:
            dy2 = dy2.to(gate.dtype)
        gs = 1.0 / (1.0 - ctx.p) if ctx.act == 2 else 1.0
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(x2.shape, device=x2.device, dtype=x2.dtype)
        want_db = ctx.has_bias and ctx.needs_input_grad[2]
        if want_db:
            db = _grad_buffer(ctx.bias_param, (w.shape[0],), w.device)
        if ctx.needs_input_grad[1]:
            dw = _grad_buffer(w, w.shape, w.device)
        elif want_db:
            _ops().colsum(dy2, gate, gs, db, 0.0)
        if dx is not None or dw is not None:
            # dX = gate(dY) W and dW = gate(dY)^T X (+ db as the GEMM's ones column): one launch
            _ops().linear_bwd(dy2, x2, w, gate, gs, dx, dw, db if dw is not None else None, _mfma())
        if dx is not None:
            dx = dx.view(*ctx.lead, x2.shape[1])
        return dx, dw, db, None, None, None, None, None, None


def linear(x, weight, bias=None, act: str = "none", p: float = 0.0, out_dtype: torch.dtype | None = None):
    """y = act(x @ W^T + b); act in {'none', 'relu', 'relu_dropout'} (dropout prob p)."""
    if act not in _ACT:
        raise ValueError(f"unknown activation {act!r}")
    if not x.is_cuda:
        y = F.linear(x, weight, bias)
        if act != "none":
            y = F.relu(y)
        if act == "relu_dropout":
            y = F.dropout(y, p, True)
        return y
    a = _ACT[act]
    if a == 2 and p == 0.0:
        a = 1
    seed, off, dev = default_state.next() if a == 2 else (0, 0, None)
    od = out_dtype or _act_dtype(x)
    return _Linear.apply(x, weight, bias, a, float(p), seed, off, dev, od)


# ----------------------------------------------------------- softmax/loss ----
class _LogSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        y = torch.empty(x.shape, device=x.device, dtype=torch.float32)
        _ops().log_softmax_fwd(x, y)
        ctx.save_for_backward(y)
        ctx.xdtype = x.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dx = torch.empty(y.shape, device=y.device, dtype=ctx.xdtype)
        _ops().log_softmax_bwd(dy.contiguous().float(), y, dx)
        return dx


def log_softmax(x, dim: int = 1):
    if not x.is_cuda:
        return F.log_softmax(x, dim=dim)
    if dim not in (1, -1) or x.dim() != 2:
        raise ValueError("log_softmax kernel supports 2-D inputs over dim 1")
    return _LogSoftmax.apply(x)


_RED = {"none": 0, "mean": 1, "sum": 2}


class _NLL(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logp, target, reduction):
        logp = logp.contiguous().float()
        target = target.contiguous().long()
        out = torch.empty((logp.shape[0],) if reduction == 0 else (), device=logp.device, dtype=torch.float32)
        _ops().nll_fwd(logp, target, out, reduction, None)
        ctx.save_for_backward(target)
        ctx.reduction, ctx.shape = reduction, logp.shape
        return out

    @staticmethod
    def backward(ctx, gout):
        (target,) = ctx.saved_tensors
        d = torch.empty(ctx.shape, device=target.device, dtype=torch.float32)
        _ops().nll_bwd(gout.contiguous().float(), target, d, ctx.reduction)
        return d, None, None


def nll_loss(logp, target, reduction: str = "mean", size_average: bool | None = None):
    """F.nll_loss; ``size_average=False`` maps to reduction='sum' (ref src/train.py:94)."""
    if size_average is not None:
        reduction = "mean" if size_average else "sum"
    if not logp.is_cuda:
        return F.nll_loss(logp, target, reduction=reduction)
    return _NLL.apply(logp, target, _RED[reduction])


class _LogSoftmaxNLL(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, target, reduction):
        z = z.contiguous()
        target = target.contiguous().long()
        logp = torch.empty(z.shape, device=z.device, dtype=torch.float32)
        out = torch.empty((z.shape[0],) if reduction == 0 else (), device=z.device, dtype=torch.float32)
        _ops().lsm_nll_fwd(z, target, logp, out, reduction)
        ctx.save_for_backward(logp, target)
        ctx.reduction, ctx.zdtype = reduction, z.dtype
        return out

    @staticmethod
    def backward(ctx, gout):
        logp, target = ctx.saved_tensors
        dz = torch.empty(logp.shape, device=logp.device, dtype=ctx.zdtype)
        _ops().lsm_nll_bwd(gout.contiguous().float(), logp, target, dz, ctx.reduction)
        return dz, None, None


def log_softmax_nll(z, target, reduction: str = "mean"):
    """nll_loss(log_softmax(z, 1), target): one kernel each way instead of four (the modular step's
    loss on logits: ref src/model.py:22 + src/train.py:74)."""
    if not z.is_cuda:
        return F.nll_loss(F.log_softmax(z, dim=1), target, reduction=reduction)
    if z.dim() != 2:
        raise ValueError("log_softmax_nll expects [rows, classes] logits")
    return _LogSoftmaxNLL.apply(z, target, _RED[reduction])


# the fused head's loss words (fixed-point sum + arrival count, int64), one per head weight (zero between launches;
# launches of one head are stream-ordered)
_head_cnt: dict[int, tuple[weakref.ref, torch.Tensor]] = {}


def _head_counter(w: torch.Tensor) -> torch.Tensor:
    hit = _head_cnt.get(id(w))
    if hit is None or hit[0]() is not w or hit[1].device != w.device:
        for k in [k for k, (r, _) in _head_cnt.items() if r() is None]:
            del _head_cnt[k]
        hit = (weakref.ref(w), torch.zeros(1, device=w.device, dtype=torch.int64))
        _head_cnt[id(w)] = hit
    return hit[1]


class _LinearLogSoftmaxNLL(torch.autograd.Function):
    """nll(log_softmax(x W^T + b)): ONE forward launch (the GEMM's epilogue computes the row-wise
    log_softmax and the NLL, the per-tile sums handed to the last tile) and ONE backward launch whose
    paired GEMMs read dz = g * (exp(logp) - onehot) straight from the kept log-probs (no logits or
    dz tensors, no separate loss kernels)."""

    @staticmethod
    def forward(ctx, x, w, b, target, reduction):
        x2 = x.contiguous()
        target = target.contiguous().long()
        logp = torch.empty((x2.shape[0], w.shape[0]), device=x.device, dtype=torch.float32)
        out = torch.empty((), device=x.device, dtype=torch.float32)
        if _ops().linear_lsm_nll_ok(x2, w):  # GEMM + log_softmax + NLL in one launch
            part = torch.empty((x2.shape[0] + 15) // 16, device=x.device, dtype=torch.float32)
            _ops().linear_lsm_nll_fwd(x2, w, b, target, logp, out, part, _head_counter(w), reduction, _mfma())
        else:
            z = torch.empty(logp.shape, device=x.device, dtype=torch.float32)
            _ops().gemm(x2, w.t(), z, b, 1.0, 0.0, 0, 0.0, 0, 0, None, None, 1.0, _mfma())
            _ops().lsm_nll_fwd(z, target, logp, out, reduction)
        ctx.save_for_backward(x2, w, logp, target)
        ctx.reduction, ctx.has_bias, ctx.bias_param = reduction, b is not None, b
        return out

    @staticmethod
    def backward(ctx, gout):
        x2, w, logp, target = ctx.saved_tensors
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(x2.shape, device=x2.device, dtype=x2.dtype)
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            dw = _grad_buffer(w, w.shape, w.device)
            if ctx.has_bias:
                db = _grad_buffer(ctx.bias_param, (w.shape[0],), w.device)
        div = float(logp.shape[0]) if ctx.reduction == 1 else 1.0
        _ops().linear_bwd(logp, x2, w, None, 1.0, dx, dw, db, _mfma(), target, gout.contiguous().float(), div)
        return dx, dw if ctx.needs_input_grad[1] else None, db if ctx.needs_input_grad[2] else None, None, None


def linear_log_softmax_nll(x, weight, bias, target, reduction: str = "mean"):
    """nll_loss(log_softmax(linear(x, weight, bias), 1), target) -- a classifier head and its loss
    (ref src/model.py:21-22 + src/train.py:74) as one forward and one backward launch.  reduction:
    'mean' or 'sum'."""
    if not x.is_cuda:
        return F.nll_loss(F.log_softmax(F.linear(x, weight, bias), dim=1), target, reduction=reduction)
    if reduction not in ("mean", "sum"):
        raise ValueError("linear_log_softmax_nll supports reduction 'mean' or 'sum'")
    return _LinearLogSoftmaxNLL.apply(x, weight, bias, target, _RED[reduction])


def cross_entropy(x, target, reduction: str = "mean"):
    """nn.CrossEntropyLoss: log_softmax then NLL (idempotent on log-probs, ref src/train_dist.py:67)."""
    return log_softmax_nll(x, target, reduction)


def accuracy_count(logp: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Number of argmax hits, kept on device (no host sync)."""
    return (logp.argmax(dim=1) == target).sum()


_DT_CODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


class _MlpHeadNLL(torch.autograd.Function):
    """nll(log_softmax(act(x W1^T + b1) W2^T + b2)): fc1 with its ReLU / dropout and the classifier
    head + loss in ONE forward launch (h kept in LDS between them, written once for the backward);
    the backward is the two layers' own: the head's paired GEMMs from the log-probs, then fc1's
    (gate = h), so gradients are those of linear() + linear_log_softmax_nll()."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, target, act, p, seed, off, dev, reduction):
        x2 = x.contiguous()
        target = target.contiguous().long()
        M = x2.shape[0]
        h = torch.empty((M, w1.shape[0]), device=x.device, dtype=_act_dtype(x2))
        logp = torch.empty((M, w2.shape[0]), device=x.device, dtype=torch.float32)
        out = torch.empty((), device=x.device, dtype=torch.float32)
        part = torch.empty((M + 15) // 16, device=x.device, dtype=torch.float32)
        _ops().mlp_head_fwd(x2, w1, b1, act, p, seed, off, dev, h, w2, b2, target, logp, out, part,
                            _head_counter(w2), reduction, _mfma())
        ctx.save_for_backward(x2, w1, h, w2, logp, target)
        ctx.act, ctx.p, ctx.reduction = act, p, reduction
        ctx.b1, ctx.b2 = b1, b2
        return out

    @staticmethod
    def backward(ctx, gout):
        x2, w1, h, w2, logp, target = ctx.saved_tensors
        need = ctx.needs_input_grad
        mf = _mfma()
        div = float(logp.shape[0]) if ctx.reduction == 1 else 1.0
        gs = 1.0 / (1.0 - ctx.p) if ctx.act == 2 else 1.0
        if ctx.act and all(need[:5]) and ctx.b1 is not None and ctx.b2 is not None:
            # the whole head's backward in one launch when it fits (dh recomputed per block, never stored)
            dx = torch.empty(x2.shape, device=x2.device, dtype=x2.dtype)
            dw1, db1 = _grad_buffer(w1, w1.shape, w1.device), _grad_buffer(ctx.b1, (w1.shape[0],), w1.device)
            dw2, db2 = _grad_buffer(w2, w2.shape, w2.device), _grad_buffer(ctx.b2, (w2.shape[0],), w2.device)
            if _ops().mlp_head_bwd(logp, target, gout.contiguous().float(), div, h, x2, w1, w2, gs, dx, dw1, db1,
                                   dw2, db2, mf):
                return dx, dw1, db1, dw2, db2, None, None, None, None, None, None, None
        # the head (linear_log_softmax_nll's backward): dh, dW2, db2 from the kept log-probs
        dh = torch.empty(h.shape, device=h.device, dtype=h.dtype) if (need[0] or need[1] or need[2]) else None
        dw2 = db2 = None
        if need[3] or (ctx.b2 is not None and need[4]):
            dw2 = _grad_buffer(w2, w2.shape, w2.device)
            if ctx.b2 is not None:
                db2 = _grad_buffer(ctx.b2, (w2.shape[0],), w2.device)
        _ops().linear_bwd(logp, h, w2, None, 1.0, dh, dw2, db2, mf, target, gout.contiguous().float(), div)
        # fc1 (linear()'s backward, gate = h)
        dx = dw1 = db1 = None
        if dh is not None:
            if need[0]:
                dx = torch.empty(x2.shape, device=x2.device, dtype=x2.dtype)
            if need[1] or (ctx.b1 is not None and need[2]):
                dw1 = _grad_buffer(w1, w1.shape, w1.device)
                if ctx.b1 is not None:
                    db1 = _grad_buffer(ctx.b1, (w1.shape[0],), w1.device)
            _ops().linear_bwd(dh, x2, w1, h if ctx.act else None, gs, dx, dw1, db1, mf)
        return (dx, dw1 if need[1] else None, db1 if need[2] else None, dw2 if need[3] else None,
                db2 if need[4] else None, None, None, None, None, None, None, None)


def mlp_head_nll(x, w1, b1, w2, b2, target, act: str = "relu", p: float = 0.0, reduction: str = "mean"):
    """nll_loss(log_softmax(linear(linear(x, w1, b1, act, p), w2, b2), 1), target) -- an MLP classifier
    head and its loss (ref src/model.py:19-22 + src/train.py:74): one forward launch when the shapes fit
    (fc1 width <= 64, <= 16 classes, a small batch), else linear() + linear_log_softmax_nll()."""
    if reduction not in ("mean", "sum"):
        raise ValueError("mlp_head_nll supports reduction 'mean' or 'sum'")
    if act not in _ACT:
        raise ValueError(f"unknown activation {act!r}")
    if not x.is_cuda:
        return linear_log_softmax_nll(linear(x, w1, b1, act, p), w2, b2, target, reduction)
    a = _ACT[act]
    if a == 2 and p == 0.0:
        a = 1
    x2 = x.reshape(-1, x.shape[-1])
    if x2.dtype not in (torch.bfloat16, torch.float16, torch.float32) or not _ops().mlp_head_ok(
            x2, w1, w2, _DT_CODE[_act_dtype(x2)], _mfma()):
        return linear_log_softmax_nll(linear(x, w1, b1, act, p), w2, b2, target, reduction)
    seed, off, dev = default_state.next() if a == 2 else (0, 0, None)  # (linear()'s draw, same order)
    return _MlpHeadNLL.apply(x2, w1, b1, w2, b2, target, a, float(p), seed, off, dev, _RED[reduction])

