"""The modular step's fused launches against their unfused equivalents (bitwise where the same
arithmetic runs) and against a plain PyTorch fp32 reference:

* conv2d_bwd: dW, db and dX of a pool-fused conv in ONE launch, the pooled gradient expanded in
  the kernels' staging == maxpool_relu_bwd + conv2d_wgrad + conv2d_dgrad (bitwise);
* conv2d_fwd with the Dropout2d mask drawn in its epilogue == channel_mask + conv2d_fwd (bitwise);
* linear_bwd: dX and dW (+ db) in one launch == the two gemm launches (bitwise);
* log_softmax_nll: one kernel each way == torch's log_softmax + nll_loss in fp32;
* the classifier head + loss (linear_log_softmax_nll): its backward GEMMs read dz from the kept
  log-probs == lsm_nll_bwd + linear_bwd (bitwise), and Net's fused head == its log-probs + nll_loss.
"""
import pytest
import torch
import torch.nn.functional as F

from csed_514_project_distributed_training_using_pytorch_amd import ops
from csed_514_project_distributed_training_using_pytorch_amd.ops import _native
from csed_514_project_distributed_training_using_pytorch_amd.ops.functional import wgrad_workspace_elems

pytestmark = pytest.mark.gpu
DEV = "cuda"
MF = {torch.bfloat16: 1, torch.float16: 2, torch.float32: 0}


@pytest.fixture(autouse=True, scope="module")
def _native_loaded():
    _native.require()
    yield


def _pooled_fwd(x, w, b, dt, scale):
    N, OC = x.shape[0], w.shape[0]
    OH, OW = x.shape[2] - w.shape[2] + 1, x.shape[3] - w.shape[3] + 1
    y = torch.empty(N, OC, OH // 2, OW // 2, device=DEV, dtype=dt)
    idx = torch.empty(y.shape, device=DEV, dtype=torch.uint8)
    _native.ops().conv2d_fwd(x, w, b, y, 0, idx, scale, 2, MF[dt])
    return y, idx


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("shape,with_dx", [((64, 10, 12, 12, 20), True), ((5, 1, 28, 28, 10), False),
                                           ((3, 4, 10, 14, 16), True)])
def test_conv_bwd_pooled_matches_unfused_bitwise(dt, shape, with_dx):
    N, C, H, W, OC = shape
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(N, C, H, W, device=DEV, generator=g).to(dt)
    w = torch.randn(OC, C, 5, 5, device=DEV, generator=g) * 0.2
    b = torch.randn(OC, device=DEV, generator=g) * 0.1
    scale = (torch.rand(N * OC, device=DEV, generator=g) > 0.5).float() * 2.0
    y, idx = _pooled_fwd(x, w, b, dt, scale)
    dy = torch.randn(y.shape, device=DEV, generator=g).to(dt)
    ws = torch.empty(wgrad_workspace_elems(N, C, 5, 5, OC), device=DEV)
    o = _native.ops()
    # fused: one launch (+ reduce), pooled dy expanded on load
    dw1, db1 = torch.empty_like(w), torch.empty_like(b)
    dx1 = torch.empty_like(x) if with_dx else None
    o.conv2d_bwd(x, dy, w, dw1, db1, ws, dx1, 0, idx, y, scale, MF[dt])
    # unfused: dL/dconv materialised, then the weight and data gradients
    dconv = torch.empty(N, OC, H - 4, W - 4, device=DEV, dtype=dt)
    o.maxpool_relu_bwd(dy, y, idx, scale, dconv, 2)
    dw2, db2 = torch.empty_like(w), torch.empty_like(b)
    o.conv2d_wgrad(x, dconv, dw2, db2, ws, 0, MF[dt], 0.0)
    assert torch.equal(dw1, dw2) and torch.equal(db1, db2)
    if with_dx:
        dx2 = torch.empty_like(x)
        o.conv2d_dgrad(dconv, w, dx2, 0, MF[dt])
        assert torch.equal(dx1, dx2)
    # and the fp32 reference of the backward, from the kernel forward's own argmax / gate (a
    # reference forward in fp32 would pick other maxima at near-ties of the 16-bit one)
    dconv_ref = _unpool_ref(dy, idx, y, scale)
    xf, wf = x.float().cpu(), w.to(dt).float().cpu()
    refs = [(dw1, torch.nn.grad.conv2d_weight(xf, w.shape, dconv_ref), "dw"), (db1, dconv_ref.sum((0, 2, 3)), "db")]
    if with_dx:
        refs.append((dx1, torch.nn.grad.conv2d_input(x.shape, wf, dconv_ref), "dx"))
    tol = 1e-4 if dt == torch.float32 else 3e-2
    for got, ref, name in refs:
        err = (got.float().cpu() - ref).abs().max().item()
        assert err <= tol * max(ref.abs().max().item(), 1e-6), f"{name}: {err:.3e}"


def _unpool_ref(dy, idx, y, scale):
    """dL/dconv of relu(maxpool2(conv) * scale) from the pooled gradient, the argmax bytes and the
    pooled output (maxpool_relu_bwd's rule) in fp32 on the CPU."""
    N, OC, PH, PW = dy.shape
    sel = torch.arange(4).view(1, 1, 1, 1, 4)
    keep = (idx.long().cpu().unsqueeze(-1) == sel) & (y.float().cpu() > 0).unsqueeze(-1)
    val = (dy.float().cpu() * scale.cpu().view(N, OC, 1, 1)).unsqueeze(-1) * keep
    return val.view(N, OC, PH, PW, 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(N, OC, 2 * PH, 2 * PW)


@pytest.mark.parametrize("N,OC", [(64, 20), (5, 80), (1100, 20)])
def test_conv_fwd_in_kernel_dropout2d_matches_channel_mask(N, OC):
    """OC = 80: channels past the first 64 (their bias / scale from the staged epilogue operands);
    N = 1100: the narrow persistent-block form (work items walked by fewer blocks)."""
    C = 10
    g = torch.Generator(device=DEV).manual_seed(4)
    x = torch.randn(N, C, 12, 12, device=DEV, generator=g).to(torch.bfloat16)
    w = torch.randn(OC, C, 5, 5, device=DEV, generator=g) * 0.2
    b = torch.randn(OC, device=DEV, generator=g) * 0.1
    off_dev = torch.tensor([5], device=DEV, dtype=torch.long)
    o = _native.ops()
    sc_ref = torch.empty(N * OC, device=DEV)
    o.channel_mask(sc_ref, 0.5, 1234, 7, off_dev)
    y_ref, idx_ref = _pooled_fwd(x, w, b, torch.bfloat16, sc_ref)
    y = torch.empty_like(y_ref)
    idx = torch.empty_like(idx_ref)
    sc = torch.full((N * OC,), -1.0, device=DEV)
    o.conv2d_fwd(x, w, b, y, 0, idx, None, 2, 1, 0.5, 1234, 7, off_dev, sc)
    assert torch.equal(sc, sc_ref)
    assert torch.equal(y, y_ref) and torch.equal(idx, idx_ref)
    assert 0.3 < (sc_ref == 0).float().mean().item() < 0.7


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("act,mio", [(2, (64, 50, 320)), (0, (64, 10, 50)), (1, (37, 70, 45)), (0, (512, 10, 50))])
def test_linear_bwd_pair_matches_two_gemms(dt, act, mio):
    M, O, I = mio
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(M, I, device=DEV, generator=g).to(dt)
    w = torch.randn(O, I, device=DEV, generator=g) * 0.1
    dy = torch.randn(M, O, device=DEV, generator=g).to(dt if act else torch.float32)
    gate = torch.randn(M, O, device=DEV, generator=g).to(dt) if act else None
    gs = 2.0 if act == 2 else 1.0
    o = _native.ops()
    dx1, dw1, db1 = torch.empty_like(x), torch.empty_like(w), torch.empty(O, device=DEV)
    o.linear_bwd(dy, x, w, gate, gs, dx1, dw1, db1, MF[dt])
    dx2, dw2, db2 = torch.empty_like(x), torch.empty_like(w), torch.empty(O, device=DEV)
    o.gemm(dy, w, dx2, None, 1.0, 0.0, 0, 0.0, 0, 0, None, gate, gs, MF[dt])
    o.gemm(dy.t(), x, dw2, None, 1.0, 0.0, 0, 0.0, 0, 0, None, gate.t() if gate is not None else None, gs, MF[dt], db2)
    assert torch.equal(dx1, dx2) and torch.equal(dw1, dw2) and torch.equal(db1, db2)
    # fp32 reference
    d = dy.float() if gate is None else torch.where(gate.float() > 0, dy.float() * gs, torch.zeros_like(dy.float()))
    tol = 1e-4 if dt == torch.float32 else 3e-2
    for got, ref in ((dx1, d @ w.to(dt).float()), (dw1, d.t() @ x.float()), (db1, d.sum(0))):
        assert (got.float() - ref).abs().max().item() <= tol * max(ref.abs().max().item(), 1e-6)


@pytest.mark.parametrize("red", ["mean", "sum", "none"])
@pytest.mark.parametrize("rows", [64, 8, 1000])
def test_log_softmax_nll_matches_torch(red, rows):
    g = torch.Generator(device=DEV).manual_seed(6)
    z = (torch.randn(rows, 10, device=DEV, generator=g) * 3).requires_grad_(True)
    t = torch.randint(0, 10, (rows,), device=DEV, generator=g)
    loss = ops.log_softmax_nll(z, t, red)
    zr = z.detach().cpu().double().requires_grad_(True)
    lr = F.nll_loss(F.log_softmax(zr, 1), t.cpu(), reduction=red)
    assert torch.allclose(loss.detach().cpu().double(), lr.detach(), rtol=2e-6, atol=1e-6)
    gout = torch.randn(loss.shape, device=DEV, generator=g)
    loss.backward(gout)
    lr.backward(gout.cpu().double())
    assert torch.allclose(z.grad.cpu().double(), zr.grad, rtol=1e-4, atol=1e-6)  # (__expf / __logf, fp32)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("red", [1, 2])
def test_loss_head_backward_matches_unfused_bitwise(dt, red):
    """linear_bwd reading dz from the log-probs == lsm_nll_bwd's dz fed to linear_bwd."""
    B, C, I = 64, 10, 50
    g = torch.Generator(device=DEV).manual_seed(8)
    h = torch.randn(B, I, device=DEV, generator=g).to(dt)
    w = torch.randn(C, I, device=DEV, generator=g) * 0.1
    logp = torch.log_softmax(torch.randn(B, C, device=DEV, generator=g) * 2, 1)
    t = torch.randint(0, C, (B,), device=DEV, generator=g)
    gout = torch.tensor(1.7, device=DEV)
    o = _native.ops()
    dx1, dw1, db1 = torch.empty_like(h), torch.empty_like(w), torch.empty(C, device=DEV)
    o.linear_bwd(logp, h, w, None, 1.0, dx1, dw1, db1, MF[dt], t, gout, float(B) if red == 1 else 1.0)
    dz = torch.empty(B, C, device=DEV)
    o.lsm_nll_bwd(gout, logp, t, dz, red)
    dx2, dw2, db2 = torch.empty_like(h), torch.empty_like(w), torch.empty(C, device=DEV)
    o.linear_bwd(dz, h, w, None, 1.0, dx2, dw2, db2, MF[dt])
    assert torch.equal(dx1, dx2) and torch.equal(dw1, dw2) and torch.equal(db1, db2)


def test_net_fused_head_matches_log_probs_path():
    """Net's fused classifier head + loss (what the modular engine runs) == nll_loss on its log-probs."""
    from csed_514_project_distributed_training_using_pytorch_amd.models import Net

    torch.manual_seed(1)
    net = Net().to(DEV).train()
    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.rand(64, 1, 28, 28, device=DEV, generator=g)
    t = torch.randint(0, 10, (64,), device=DEV, generator=g)
    grads = []
    for fused in (True, False):
        ops.rng.default_state.reset_offset()  # (the same dropout masks in both passes)
        net.zero_grad(set_to_none=True)
        loss = net(x, target=t) if fused else ops.nll_loss(net(x), t)
        loss.backward()
        grads.append((loss.detach(), [p.grad.clone() for p in net.parameters()]))
    (l1, g1), (l2, g2) = grads
    assert torch.allclose(l1, l2, rtol=1e-6, atol=1e-6)
    for a, b in zip(g1, g2):
        assert (a - b).abs().max().item() <= 1e-2 * max(b.abs().max().item(), 1e-6)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,red", [(64, 1), (37, 2), (1000, 1)])
def test_head_forward_matches_gemm_then_loss(dt, rows, red):
    """The classifier head's one-launch forward (log_softmax + NLL in the GEMM epilogue, per-tile
    sums handed to the last tile) == gemm + lsm_nll_fwd, over repeated launches (the arrival
    counter re-arms itself)."""
    g = torch.Generator(device=DEV).manual_seed(9)
    x = torch.randn(rows, 50, device=DEV, generator=g).to(dt)
    w = torch.randn(10, 50, device=DEV, generator=g) * 0.3
    b = torch.randn(10, device=DEV, generator=g)
    t = torch.randint(0, 10, (rows,), device=DEV, generator=g)
    o = _native.ops()
    assert o.linear_lsm_nll_ok(x, w)
    z = torch.empty(rows, 10, device=DEV)
    o.gemm(x, w.t(), z, b, 1.0, 0.0, 0, 0.0, 0, 0, None, None, 1.0, MF[dt])
    lp_ref, out_ref = torch.empty_like(z), torch.empty((), device=DEV)
    o.lsm_nll_fwd(z, t, lp_ref, out_ref, red)
    cnt = torch.zeros(1, device=DEV, dtype=torch.int64)
    part = torch.empty((rows + 15) // 16, device=DEV)
    for _ in range(3):
        lp, out = torch.full_like(z, 7.0), torch.full((), 7.0, device=DEV)
        o.linear_lsm_nll_fwd(x, w, b, t, lp, out, part, cnt, red, MF[dt])
        torch.testing.assert_close(lp, lp_ref, rtol=0, atol=2e-6)
        torch.testing.assert_close(out, out_ref, rtol=2e-6, atol=2e-6)
        assert int(cnt.item()) == 0


@pytest.mark.parametrize("rows", [4096, 20000])
def test_head_large_batch_fallback(rows):
    """Past the small-GEMM path (K = batch > 1024 in dW, more than 1024 row tiles) the head runs
    gemm + loss kernel forward and materialises dz backward; same values as the fp32 reference."""
    g = torch.Generator(device=DEV).manual_seed(10)
    x = torch.randn(rows, 50, device=DEV, generator=g).to(torch.bfloat16).requires_grad_(True)
    w = (torch.randn(10, 50, device=DEV, generator=g) * 0.3).requires_grad_(True)
    b = torch.randn(10, device=DEV, generator=g).requires_grad_(True)
    t = torch.randint(0, 10, (rows,), device=DEV, generator=g)
    loss = ops.linear_log_softmax_nll(x, w, b, t)
    loss.backward()
    xr = x.detach().float().cpu().requires_grad_(True)
    wr = w.detach().to(torch.bfloat16).float().cpu().requires_grad_(True)
    br = b.detach().cpu().requires_grad_(True)
    lr = F.nll_loss(F.log_softmax(F.linear(xr, wr, br), 1), t.cpu())
    lr.backward()
    assert abs(loss.item() - lr.item()) <= 1e-3 * abs(lr.item())
    for got, ref in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert (got.float().cpu() - ref).abs().max().item() <= 3e-2 * max(ref.abs().max().item(), 1e-6)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,act,red", [(64, "relu_dropout", "mean"), (37, "relu", "sum"),
                                          (200, "relu_dropout", "mean"), (8, "relu_dropout", "sum")])
def test_mlp_head_matches_two_launch_path_bitwise(dt, rows, act, red):
    """mlp_head_nll (fc1 + relu / dropout + fc2 + log_softmax + NLL in ONE launch, h kept in LDS) ==
    linear() + linear_log_softmax_nll() bitwise: the same K split and combine order for fc1, the same
    dropout draw, the head's K-steps and epilogue as the small GEMM's; the backward is theirs."""
    from csed_514_project_distributed_training_using_pytorch_amd.ops import functional as fn

    prev = fn.compute_dtype()
    fn.set_compute_dtype(dt)
    try:
        g = torch.Generator(device=DEV).manual_seed(11)
        x0 = torch.randn(rows, 320, device=DEV, generator=g).relu().to(dt if dt != torch.float32 else torch.float32)
        w1 = torch.randn(50, 320, device=DEV, generator=g) * 0.05
        b1 = torch.randn(50, device=DEV, generator=g) * 0.1
        w2 = torch.randn(10, 50, device=DEV, generator=g) * 0.2
        b2 = torch.randn(10, device=DEV, generator=g) * 0.1
        t = torch.randint(0, 10, (rows,), device=DEV, generator=g)
        assert _native.ops().mlp_head_ok(x0, w1, w2, fn._DT_CODE[fn._act_dtype(x0)], MF[dt])
        res = []
        for fused in (True, False):
            ops.rng.default_state.reset_offset()  # (the same dropout masks in both passes)
            leaves = [v.detach().clone().requires_grad_(True) for v in (x0, w1, b1, w2, b2)]
            x, a1, c1, a2, c2 = leaves
            if fused:
                loss = ops.mlp_head_nll(x, a1, c1, a2, c2, t, act=act, p=0.5, reduction=red)
            else:
                loss = ops.linear_log_softmax_nll(ops.linear(x, a1, c1, act=act, p=0.5), a2, c2, t, reduction=red)
            loss.backward()
            res.append((loss.detach(), [v.grad for v in leaves]))
        (l1, g1), (l2, g2) = res
        assert torch.equal(l1, l2), (l1.item(), l2.item())
        for a, b in zip(g1, g2):
            assert torch.equal(a, b)
        # and against an fp32 reference of the same masks (loose: 16-bit operands)
        if act == "relu":
            lr = F.nll_loss(F.log_softmax(F.linear(F.relu(F.linear(x0.float(), w1, b1)), w2, b2), 1), t, reduction=red)
            assert abs(l1.item() - lr.item()) <= 2e-2 * max(abs(lr.item()), 1.0)
    finally:
        fn.set_compute_dtype(prev)


def test_mlp_head_repeated_launches_rearm_counter():
    """The fused MLP head's loss hand-off counter is zero again after every launch."""
    g = torch.Generator(device=DEV).manual_seed(12)
    x = torch.randn(64, 320, device=DEV, generator=g).to(torch.bfloat16)
    w1, w2 = torch.randn(50, 320, device=DEV, generator=g) * 0.05, torch.randn(10, 50, device=DEV, generator=g) * 0.2
    t = torch.randint(0, 10, (64,), device=DEV, generator=g)
    first = None
    for _ in range(4):
        loss = ops.mlp_head_nll(x, w1, None, w2, None, t, act="relu")
        first = loss if first is None else first
        assert torch.equal(loss, first)
    from csed_514_project_distributed_training_using_pytorch_amd.ops import functional as fn
    assert int(fn._head_counter(w2).item()) == 0


@pytest.mark.parametrize("head", ["linear", "mlp"])
def test_head_loss_recovers_after_nonfinite_and_huge_losses(head):
    """A NaN logit, then huge losses in many tiles, then a finite batch: the first two report a
    non-finite loss, the finite batch's loss is right again (the hand-off word never carried into its
    arrival count) and the word is re-armed to 0 after each launch."""
    from csed_514_project_distributed_training_using_pytorch_amd.ops import functional as fn

    g = torch.Generator(device=DEV).manual_seed(21)
    M = 256  # 16 tiles
    x = torch.randn(M, 50, device=DEV, generator=g)
    w = torch.randn(10, 50, device=DEV, generator=g) * 0.2
    b = torch.zeros(10, device=DEV)
    t = torch.randint(0, 10, (M,), device=DEV, generator=g)

    def loss_of(xx, bb=b):
        if head == "linear":
            return ops.linear_log_softmax_nll(xx, w, bb, t, reduction="sum")
        return ops.mlp_head_nll(xx.to(torch.bfloat16), w1, None, w, bb, t, act="relu", reduction="sum")

    w1 = torch.eye(50, device=DEV)  # (mlp: relu(x) feeds the head)
    bad = b.clone()
    bad[7] = float("nan")  # (a NaN logit in every row; the fc1 ReLU would turn a NaN input into 0)
    assert not torch.isfinite(loss_of(x, bad)).item()
    assert int(fn._head_counter(w).item()) == 0
    huge = x * 1e8  # every tile's sum far above the fixed-point range
    assert not torch.isfinite(loss_of(huge)).item()
    assert int(fn._head_counter(w).item()) == 0
    got = loss_of(x).item()
    xr = x if head == "linear" else torch.relu(x.to(torch.bfloat16).float())
    want = F.nll_loss(F.log_softmax(xr @ w.t() + b, 1), t, reduction="sum").item()
    assert abs(got - want) <= 2e-2 * abs(want), (got, want)
    assert int(fn._head_counter(w).item()) == 0


def _net_with_destinations():
    """Net on the GPU with its gradients registered into a flat buffer (as ModularTrainer does):
    the only configuration in which the conv weight-gradient reduce is deferred."""
    from csed_514_project_distributed_training_using_pytorch_amd.models import Net
    from csed_514_project_distributed_training_using_pytorch_amd.utils.flat import FlatParams

    torch.manual_seed(1)
    net = Net().to(DEV).train()
    flat = FlatParams(list(net.parameters()))
    for i, p in enumerate(flat.params):
        ops.set_grad_destination(p, flat.grad_view(i))
    g = torch.Generator(device=DEV).manual_seed(13)
    x = torch.rand(64, 1, 28, 28, device=DEV, generator=g)
    t = torch.randint(0, 10, (64,), device=DEV, generator=g)
    return net, flat, x, t


def _drop_destinations(flat):
    for p in flat.params:
        ops.set_grad_destination(p, None)


def _backward(net, x, t):
    ops.rng.default_state.reset_offset()
    net(x, target=t).backward()


def test_deferred_wgrad_reduce_matches_immediate_bitwise():
    """conv2's weight-gradient reduce carried by conv1's backward launch (and the end-of-backward flush)
    == every conv reducing in its own launch, bitwise; nothing stays pending after backward; a
    parameter watched by a post-accumulate-grad hook (a DDP reducer's) is reduced before its hook."""
    from csed_514_project_distributed_training_using_pytorch_amd.ops import functional as fn

    net, flat, x, t = _net_with_destinations()
    res = []
    try:
        for defer in (True, False):
            fn.set_defer_wgrad_reduce(defer)
            net.zero_grad(set_to_none=True)
            _backward(net, x, t)
            assert fn.pending_reduce_count() == 0
            assert flat.grads_are_views()  # (adopted: written in place)
            res.append([p.grad.clone() for p in net.parameters()])
        for a, b in zip(*res):
            assert torch.equal(a, b)
        fn.set_defer_wgrad_reduce(True)
        seen = {}

        def hook(p):
            seen["g"] = p.grad.clone()

        hk = net.conv2.weight.register_post_accumulate_grad_hook(hook)
        try:
            net.zero_grad(set_to_none=True)
            _backward(net, x, t)
        finally:
            hk.remove()
        assert torch.equal(seen["g"], res[1][2])  # (conv2.weight: its final gradient inside the hook)
    finally:
        fn.set_defer_wgrad_reduce(True)
        _drop_destinations(flat)


def test_deferred_wgrad_reduce_with_zeroed_grads_and_accumulation():
    """Deferral on, .grad NOT None (FusedSGD.zero_grad keeps flat views; a second backward without
    zero_grad): AccumulateGrad adds dW as soon as the conv backward returns, so the reduce must not
    be deferred -- conv gradients equal the set_to_none step's, and twice them after two backwards."""
    from csed_514_project_distributed_training_using_pytorch_amd.ops import functional as fn
    from csed_514_project_distributed_training_using_pytorch_amd.optim import FusedSGD

    net, flat, x, t = _net_with_destinations()
    try:
        fn.set_defer_wgrad_reduce(True)
        net.zero_grad(set_to_none=True)
        _backward(net, x, t)
        ref = [p.grad.clone() for p in net.parameters()]
        opt = FusedSGD(list(net.parameters()), lr=0.01, momentum=0.5, flat=flat)
        opt.zero_grad()  # flat.grad zeroed, .grad = the flat views (not None)
        assert all(p.grad is not None for p in net.parameters())
        _backward(net, x, t)
        assert fn.pending_reduce_count() == 0
        for a, p in zip(ref, net.parameters()):
            assert torch.equal(p.grad, a)
        _backward(net, x, t)  # no zero_grad: accumulates
        for a, p in zip(ref, net.parameters()):
            assert torch.equal(p.grad, 2 * a)
    finally:
        fn.set_defer_wgrad_reduce(True)
        _drop_destinations(flat)


@pytest.mark.parametrize("defer", [True, False])
def test_shared_weights_with_destinations_match_cpu(defer):
    """A conv and a linear each applied twice in one forward, gradients registered into a flat buffer
    (ModularTrainer's setup): every use's dW must be summed, not written into one shared buffer --
    compared with the same model on the CPU (fp32 kernels, so the tolerance is the fp32 one)."""
    from csed_514_project_distributed_training_using_pytorch_amd.ops import functional as fn
    from csed_514_project_distributed_training_using_pytorch_amd.utils.flat import FlatParams

    torch.manual_seed(3)
    conv = torch.nn.Conv2d(4, 4, 3, padding=1)
    lin = torch.nn.Linear(16, 16)
    x = torch.randn(8, 4, 4, 4)

    def model(x, c, lw, lb):
        y = ops.conv2d(ops.conv2d(x, c.weight, c.bias, padding=1), c.weight, c.bias, padding=1)
        y = y.reshape(8, 64)[:, :16].float()
        return ops.linear(ops.linear(y, lw, lb), lw, lb).float().square().sum()

    model(x, conv, lin.weight, lin.bias).backward()
    want = [p.grad.clone() for p in (conv.weight, conv.bias, lin.weight, lin.bias)]
    gconv = torch.nn.Conv2d(4, 4, 3, padding=1).to(DEV)
    glin = torch.nn.Linear(16, 16).to(DEV)
    with torch.no_grad():
        for a, b in ((gconv, conv), (glin, lin)):
            a.weight.copy_(b.weight)
            a.bias.copy_(b.bias)
    params = [gconv.weight, gconv.bias, glin.weight, glin.bias]
    flat = FlatParams(params)
    for i, p in enumerate(flat.params):
        ops.set_grad_destination(p, flat.grad_view(i))
    ops.set_compute_dtype(torch.float32)
    fn.set_defer_wgrad_reduce(defer)
    try:
        for p in params:
            p.grad = None
        model(x.to(DEV), gconv, glin.weight, glin.bias).backward()
        torch.cuda.synchronize()
        assert fn.pending_reduce_count() == 0
        for g, p in zip(want, params):
            torch.testing.assert_close(p.grad.cpu(), g, rtol=1e-4, atol=1e-4)
    finally:
        ops.set_compute_dtype(torch.bfloat16)
        fn.set_defer_wgrad_reduce(True)
        _drop_destinations(flat)


@pytest.mark.parametrize("kind", ["fwd_pool", "fwd_pool_f32in", "fwd_plain", "dgrad", "dgrad_pooled"])
def test_conv_persistent_blocks_match_per_item_launches_bitwise(kind):
    """Large batches: the conv forward / data-gradient launch runs at most 2048 persistent blocks that
    walk the (image, band) items with the weights staged once per block (conv.hip conv_fwd_kernel).
    A batch of 2100 images (items > blocks) must give the same bits as the same images launched in
    chunks of 500 (one block per item), and match an fp32 reference.  The persistent form stages an
    unpooled input by 16-byte vectors (conv_fwd_body VM; the per-item one element by element): the
    fp32-input forward (the modular conv1) and the padded data gradient cover both of its layouts."""
    g = torch.Generator(device=DEV).manual_seed(17)
    N = 2100
    o = _native.ops()
    if kind.startswith("fwd"):
        x = torch.randn(N, 1, 28, 28, device=DEV, generator=g)
        if kind != "fwd_pool_f32in":  # (the modular step's conv1 reads the fp32 input)
            x = x.to(torch.bfloat16)
        w = torch.randn(10, 1, 5, 5, device=DEV, generator=g) * 0.3
        b = torch.randn(10, device=DEV, generator=g) * 0.1
        pool = kind.startswith("fwd_pool")

        def run(xx):
            if pool:
                y = torch.empty(xx.shape[0], 10, 12, 12, device=DEV, dtype=torch.bfloat16)
                idx = torch.empty(y.shape, device=DEV, dtype=torch.uint8)
                o.conv2d_fwd(xx, w, b, y, 0, idx, None, 2, MF[torch.bfloat16])
                return y, idx
            y = torch.empty(xx.shape[0], 10, 24, 24, device=DEV, dtype=torch.bfloat16)
            o.conv2d_fwd(xx, w, b, y, 0, None, None, 0, MF[torch.bfloat16])
            return (y,)

        full = run(x)
        parts = [run(x[i:i + 500]) for i in range(0, N, 500)]
        for j, t in enumerate(full):
            assert torch.equal(t, torch.cat([p[j] for p in parts])), j
        ref = F.conv2d(x.float().cpu(), w.to(torch.bfloat16).float().cpu(), b.cpu())
        if pool:
            ref = F.relu(F.max_pool2d(ref, 2))
        err = (full[0].float().cpu() - ref).abs().max().item()
        assert err <= 3e-2 * ref.abs().max().item(), err
    else:
        w = torch.randn(20, 10, 5, 5, device=DEV, generator=g) * 0.2
        if kind == "dgrad":
            dy = torch.randn(N, 20, 8, 8, device=DEV, generator=g).to(torch.bfloat16)

            def run(d):
                dx = torch.empty(d.shape[0], 10, 12, 12, device=DEV, dtype=torch.bfloat16)
                o.conv2d_dgrad(d, w, dx, 0, MF[torch.bfloat16])
                return dx

            full = run(dy)
            parts = torch.cat([run(dy[i:i + 500]) for i in range(0, N, 500)])
            assert torch.equal(full, parts)
            ref = torch.nn.grad.conv2d_input((N, 10, 12, 12), w.to(torch.bfloat16).float().cpu(), dy.float().cpu())
            err = (full.float().cpu() - ref).abs().max().item()
            assert err <= 3e-2 * ref.abs().max().item(), err
        else:  # the pooled backward (conv2d_bwd: dgrad launch past the merged form's grid)
            x = torch.randn(N, 10, 12, 12, device=DEV, generator=g).to(torch.bfloat16)
            bb = torch.randn(20, device=DEV, generator=g) * 0.1
            scale = (torch.rand(N * 20, device=DEV, generator=g) > 0.5).float() * 2.0

            def run(xx, sc):
                y, idx = _pooled_fwd(xx, w, bb, torch.bfloat16, sc)
                dyp = torch.ones(y.shape, device=DEV, dtype=torch.bfloat16)
                ws = torch.empty(wgrad_workspace_elems(xx.shape[0], 10, 5, 5, 20), device=DEV)
                dw, db = torch.empty_like(w), torch.empty_like(bb)
                dx = torch.empty_like(xx)
                o.conv2d_bwd(xx, dyp, w, dw, db, ws, dx, 0, idx, y, sc, MF[torch.bfloat16])
                return dx

            full = run(x, scale)
            parts = torch.cat([run(x[i:i + 500], scale[i * 20:(i + 500) * 20]) for i in range(0, N, 500)])
            assert torch.equal(full, parts)


@pytest.mark.parametrize("pooled", [True, False])
def test_conv_wgrad_staging_depth_bitwise(pooled):
    """Large batches: a weight-gradient block walks several images with the loads of the next
    PF - 1 images in flight (conv.hip conv_wgrad_body, PF > 1).  Same images, same order, same
    sums: the slab must equal the one-image-ahead form (conv_wgrad_prefetch(1)) bit for bit, and match
    an fp32 reference.  conv1's shape with a pooled dy (the modular step's conv1 backward), conv2's
    with a plain one (its materialised dL/dconv at large batch)."""
    g = torch.Generator(device=DEV).manual_seed(23)
    N = 1300  # 217 weight-gradient blocks x 6 images: per_block > 2
    o = _native.ops()
    dt = torch.bfloat16
    if pooled:
        x = torch.randn(N, 1, 28, 28, device=DEV, generator=g).to(dt)
        w = torch.randn(10, 1, 5, 5, device=DEV, generator=g) * 0.3
        b = torch.randn(10, device=DEV, generator=g) * 0.1
        scale = (torch.rand(N * 10, device=DEV, generator=g) > 0.5).float() * 2.0
        y, idx = _pooled_fwd(x, w, b, dt, scale)
        dy = torch.randn(y.shape, device=DEV, generator=g).to(dt)
    else:
        x = torch.randn(N, 10, 12, 12, device=DEV, generator=g).to(dt)
        w = torch.randn(20, 10, 5, 5, device=DEV, generator=g) * 0.2
        dy = torch.randn(N, 20, 8, 8, device=DEV, generator=g).to(dt)
    OC, C = w.shape[:2]
    ws = torch.empty(wgrad_workspace_elems(N, C, 5, 5, OC), device=DEV)
    out = {}
    prev = o.conv_wgrad_prefetch(0)
    for pf in ("1", "2"):
        o.conv_wgrad_prefetch(int(pf))
        dw, db = torch.empty_like(w), torch.empty(OC, device=DEV)
        if pooled:
            o.conv2d_bwd(x, dy, w, dw, db, ws, None, 0, idx, y, scale, MF[dt])
        else:
            o.conv2d_wgrad(x, dy, dw, db, ws, 0, MF[dt], 0.0)
        torch.cuda.synchronize()
        out[pf] = (dw, db)
    o.conv_wgrad_prefetch(prev)
    assert prev > 1, "the weight-gradient staging depth is 2 by default"
    assert torch.equal(out["1"][0], out["2"][0]) and torch.equal(out["1"][1], out["2"][1])
    dconv = _unpool_ref(dy, idx, y, scale) if pooled else dy.float().cpu()
    ref_w = torch.nn.grad.conv2d_weight(x.float().cpu(), w.shape, dconv)
    ref_b = dconv.sum((0, 2, 3))
    for got, ref in ((out["2"][0], ref_w), (out["2"][1], ref_b)):
        err = (got.float().cpu() - ref).abs().max().item()
        assert err <= 3e-2 * max(ref.abs().max().item(), 1e-6), err
