"""The fused gradient exchange of lenet_update (csrc/kernels/lenet_fused.hip ll_allreduce) and
the one-shot IPC all-reduce (csrc/comm/ipc_allreduce.hip) at world sizes 2 / 4 / 8 on ONE GPU:
loopback mode (csrc/comm ipc_open_loopback) maps the N - 1 virtual peers onto sender slots of
this rank's own receive buffer, so the kernels run their full push + poll code for N - 1 peers
and every exchange returns N x the local value.  The reference's exchange is DDP's all-reduce
of the 21,840-float gradient once per step (ref src/train_dist.py:63,83)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

N_PARAMS = 21840


def _engine(B, loopback_world=0, dtype=torch.bfloat16, n=2048, drop_p=0.5):
    from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist
    from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer
    from csed_514_project_distributed_training_using_pytorch_amd.models import Net

    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    return FusedLeNetTrainer(Net().to(dev), synthetic_mnist(n, seed=3), lr=0.05, momentum=0.5, global_batch=B,
                             compute_dtype=dtype, drop_p=drop_p, loopback_world=loopback_world)


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("B", [8, 64])
def test_loopback_exchange_returns_world_copies(world, B):
    """Integer-valued slabs through the reduce-only update with the exchange: the result is
    exactly world x the local sum, for both slot parities (4 rounds), with no timed-out wait."""
    eng = _engine(B, loopback_world=world)
    ops = torch.ops.csed
    gen = torch.Generator(device="cpu").manual_seed(5 + world + B)
    common = (eng.flat.data, eng.momentum_buf, eng.wimg, eng.lr, eng.momentum, eng.dampening, eng.weight_decay,
              eng.nesterov, eng.step_count, eng.ticket, None, None, False, None, 0, None, eng.mfma)
    for _ in range(4):
        eng.slab.copy_(torch.randint(-8, 9, eng.slab.shape, generator=gen, dtype=torch.float32))
        eng.set_fc_vectors(torch.randint(-4, 5, (eng.B, 464), generator=gen, dtype=torch.float32))
        local = torch.empty(N_PARAMS, device=eng.device)
        fused = torch.empty_like(local)
        ops.lenet_update(eng.slab, eng.grid, eng.vslab, eng.B, None, local, *common)
        ops.lenet_update(eng.slab, eng.grid, eng.vslab, eng.B, None, fused, *common, None, eng.exch.id,
                         eng.exch_timeout_s)
        torch.cuda.synchronize()
        assert torch.equal(fused, local * world)
    assert eng.comm_errors() == 0
    eng.close()


@pytest.mark.parametrize("world", [2, 8])
def test_loopback_oneshot_allreduce(world):
    """The standalone one-shot IPC all-reduce kernel (32 blocks) in loopback: world x input."""
    from csed_514_project_distributed_training_using_pytorch_amd.parallel.ipc import open_loopback_exchange

    dev = torch.device("cuda", 0)
    ar = open_loopback_exchange(dev, N_PARAMS, world, blocks=32)
    x = torch.remainder(torch.arange(N_PARAMS, device=dev, dtype=torch.float32) * 7, 61.0)
    for r in range(4):
        y = ar(x + r, torch.empty_like(x))
        torch.cuda.synchronize()
        assert torch.equal(y, (x + r) * world)
    assert ar.error() == 0
    ar.close()


def test_loopback_training_is_local_training():
    """At world 2 the loopback step scales the loss by 1/2 and sums two copies of the gradient:
    power-of-two scaling commutes with bf16 rounding, so training is bitwise the world-1
    training (graph replays + the native executor), and every exchange completed."""
    finals = []
    for world in (0, 2):
        eng = _engine(16, loopback_world=world)
        eng.set_epoch_order(torch.randperm(2048, generator=torch.Generator().manual_seed(0)))
        eng.run_steps(8, steps_per_graph=4)
        eng.run_steps(4, use_graph=False)
        torch.cuda.synchronize()
        assert eng.comm_errors() == 0
        assert eng.allreduce_kind == ("none" if world == 0 else "fused-ipc-loopback2")
        finals.append(eng.flat.data.clone())
        eng.close()
    assert torch.isfinite(finals[0]).all()
    assert torch.equal(finals[0], finals[1])


def _train16(world: int) -> torch.Tensor:
    eng = _engine(8, loopback_world=world, dtype=torch.float32)
    eng.set_epoch_order(torch.randperm(2048, generator=torch.Generator().manual_seed(1)))
    eng.run_steps(16, steps_per_graph=8)
    torch.cuda.synchronize()
    err, diag = eng.comm_errors(), eng.comm_diag()
    out = eng.flat.data.clone()
    eng.close()
    assert err == 0, f"world {world}: exchange error word {err}, first mismatch {diag}"
    return out


def test_loopback_world8_trains_close_to_local():
    """World 8 sums eight copies in rank order (not exactly 8x in fp32): close to world 1.
    Exact-fp32 kernels (with bf16 weight images a last-bit difference re-rounds an image
    element and the trajectories drift apart by ~5e-3 in 16 steps, argmax flips included).

    Three runs, so a divergence names its side: two world-1 runs must be bitwise equal (the
    step is deterministic: a difference there is the training kernel, not the exchange), and
    the world-8 run must be close to both, with the in-kernel loopback invariant clean (every
    received word bit-equal to the value pushed; a failure prints the first mismatch)."""
    local_a = _train16(0)
    world8 = _train16(8)
    local_b = _train16(0)
    assert torch.equal(local_a, local_b), "the world-1 fp32 step is not deterministic (training kernel side)"
    rel = ((world8 - local_a).norm() / local_a.norm()).item()
    assert rel < 1e-3, f"world-8 looped-back run diverged from world 1 (exchange side): rel {rel}"


def test_loopback_mismatch_is_detected():
    """The loopback invariant itself: a receive slot pre-filled with words that carry the
    next call's tag but a value nobody pushed (csrc/comm ipc_poison), with this rank's pushes
    muted, must raise the mismatch bit (not the timeout bit) and record the first bad word."""
    eng = _engine(8, loopback_world=4)
    ops = torch.ops.csed
    common = (eng.flat.data, eng.momentum_buf, eng.wimg, eng.lr, eng.momentum, eng.dampening, eng.weight_decay,
              eng.nesterov, eng.step_count, eng.ticket, None, None, False, None, 0, None, eng.mfma)
    eng.slab.fill_(1.0)
    eng.set_fc_vectors(torch.ones(eng.B, 464))
    poison = 0x7FC0BEEF  # a NaN no gradient produces
    ops.ipc_poison(eng.exch.id, 1, poison)  # fresh buffer: every workgroup's first tag is 1
    eng.exch.mute(True)
    out = torch.empty(N_PARAMS, device=eng.device)
    ops.lenet_update(eng.slab, eng.grid, eng.vslab, eng.B, None, out, *common, None, eng.exch.id,
                     eng.exch_timeout_s)
    torch.cuda.synchronize()
    err, diag = eng.comm_errors(), eng.comm_diag()
    assert err == eng.exch.ERR_MISMATCH, err
    assert diag is not None and diag["tag"] == 1 and diag["got_tag"] == 1
    assert int(diag["got_word"], 16) & 0xFFFFFFFF == poison
    assert 0 <= diag["peer_row"] < 3
    eng.exch.error(reset=True)
    assert eng.comm_diag() is None
    eng.close()
