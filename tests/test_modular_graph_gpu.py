"""The modular (per-op) engine's HIP-graph step (engine/modular.py): one replay per step must be
the same training step as the eager per-op path -- bitwise, dropout included -- with gradients
written straight into the flat buffer (no copies), a new capture per input shape (the epoch's
short last batch), and the reducer's bucketed all-reduce captured on its comm stream.
Ref: the DDP loop src/train_dist.py:80-84."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _batches(n, B, dev):
    g = torch.Generator(device=dev).manual_seed(7)
    out = []
    for i in range(n):
        b = B if i < n - 1 else B // 2  # the last one is a short batch (a second capture)
        out.append((torch.randn(b, 1, 28, 28, device=dev, generator=g).to(torch.bfloat16),
                    torch.randint(0, 10, (b,), device=dev, generator=g)))
    return out


def _train(graph: bool, batches, ctx=None, force_world=None):
    from csed_514_project_distributed_training_using_pytorch_amd.engine.modular import ModularTrainer
    from csed_514_project_distributed_training_using_pytorch_amd.models import Net

    torch.manual_seed(1)
    net = Net().cuda().train()
    tr = ModularTrainer(net, lr=0.05, momentum=0.5, ctx=ctx, graph=graph)
    if force_world:
        tr.ddp.world_size = force_world
    losses = [tr.train_batch(x, t) for x, t in batches]
    torch.cuda.synchronize()
    return tr, torch.stack(losses)


def test_graph_step_equals_eager_step():
    dev = torch.device("cuda", 0)
    batches = _batches(7, 64, dev)
    tr_e, loss_e = _train(False, batches)
    tr_g, loss_g = _train(True, batches)
    assert tr_g.use_graph and len(tr_g._graphs) == 2  # full batch + short last batch
    assert torch.equal(loss_e, loss_g)
    assert torch.equal(tr_e.flat.data, tr_g.flat.data)
    assert torch.equal(tr_e.opt.momentum_flat, tr_g.opt.momentum_flat)
    assert int(tr_g.opt.step_count.item()) == len(batches)
    # gradients were written into the flat buffer, not copied: every .grad is a view of it
    assert tr_g.flat.grads_are_views() and tr_e.flat.grads_are_views()
    # the masks differ from step to step (device step counter in the Philox offset)
    assert len(set(loss_g.tolist())) == len(batches)


def test_graph_step_follows_lr_changes():
    """An LR schedule written through opt.param_groups mid-run: the graph path must use the new lr
    (a new capture), like the eager path -- bitwise."""
    from csed_514_project_distributed_training_using_pytorch_amd.engine.modular import ModularTrainer
    from csed_514_project_distributed_training_using_pytorch_amd.models import Net

    dev = torch.device("cuda", 0)
    batches = _batches(6, 64, dev)[:5]
    res = []
    for graph in (False, True):
        torch.manual_seed(1)
        tr = ModularTrainer(Net().cuda().train(), lr=0.05, momentum=0.5, graph=graph)
        for i, (x, t) in enumerate(batches):
            if i == 2:
                tr.opt.param_groups[0]["lr"] = 0.01
            tr.train_batch(x, t)
        torch.cuda.synchronize()
        res.append(tr)
    assert len(res[1]._graphs) == 2  # one capture per lr
    assert torch.equal(res[0].flat.data, res[1].flat.data)
    assert torch.equal(res[0].opt.momentum_flat, res[1].opt.momentum_flat)


def test_graph_step_with_captured_bucketed_allreduce():
    """A one-rank RCCL process group with the reducer forced into its collective path: every
    bucket's all-reduce is captured on the comm stream inside the step graph; the result equals
    the eager step with the same collectives."""
    import os
    import types

    import torch.distributed as dist

    from csed_514_project_distributed_training_using_pytorch_amd.parallel.launch import free_port

    dev = torch.device("cuda", 0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        ctx = types.SimpleNamespace(is_distributed=True, backend="nccl")
        batches = _batches(5, 64, dev)
        tr_e, loss_e = _train(False, batches, ctx, force_world=2)
        tr_g, loss_g = _train(True, batches, ctx, force_world=2)
        assert tr_g.use_graph
        assert torch.equal(loss_e, loss_g) and torch.equal(tr_e.flat.data, tr_g.flat.data)
    finally:
        dist.destroy_process_group()
