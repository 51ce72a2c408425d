"""The gradient exchange fused into lenet_update (csrc/kernels/lenet_fused.hip,
engine/fused.py) over the IPC buffers of csrc/comm, and the RCCL fallback.

Two ranks share the box's single GPU: the handle exchange, the peer mapping,
the LL protocol (both slot parities, graph replay) and the fused engine's
data-parallel step all run for real; only the transport is local HBM rather
than xGMI.  The bootstrap process group is gloo (CPU), as on a CPU-only host.
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CSED_IPC_TIMEOUT_S="30")
        import torch.distributed as dist

        from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist
        from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer
        from csed_514_project_distributed_training_using_pytorch_amd.models import Net
        from csed_514_project_distributed_training_using_pytorch_amd.parallel.comm import DistContext
        from csed_514_project_distributed_training_using_pytorch_amd.parallel.sampler import ShardSampler

        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        ctx = DistContext(rank, world, 0, dev, "gloo")
        res = {}
        data = synthetic_mnist(2048, seed=3)

        def train(mode, key=None, split=False, gb=64):
            # fused: lenet_update exchanges with the peer itself (one kernel);
            # rccl: reduce-only update -> the process group's all-reduce (gloo here: a host sum
            # in rank order, bitwise the fused exchange's order) -> SGD kernel
            key = key or mode
            os.environ["CSED_ALLREDUCE"] = mode
            torch.manual_seed(1)
            eng = FusedLeNetTrainer(Net().to(dev), data, lr=0.05, global_batch=gb, ctx=ctx, split=split)
            res[f"split_{key}"] = eng.split
            smp = ShardSampler(2048, world, rank, shuffle=True, seed=42)
            smp.set_epoch(0)
            eng.set_epoch_order(smp.indices())
            if mode == "fused":  # the last 4 of the 12 steps through the native executor
                eng.run_steps(8, steps_per_graph=4)
                eng.run_steps(4, use_graph=False)  # (csed.LenetStepper, exchange in lenet_update)
            else:
                eng.run_steps(12, steps_per_graph=4)
            res[f"native_{key}"] = eng.stepper() is not None
            eng.step()  # one eager step after the graph replays
            torch.cuda.synchronize(dev)
            p = eng.flat.data.cpu()
            other = p.clone()
            dist.broadcast(other, src=0)
            res[f"kind_{key}"] = eng.allreduce_kind
            res[f"step_{key}"] = eng.step_kind
            res[f"params_equal_{key}"] = torch.equal(p, other)
            res[f"engine_errors_{key}"] = eng.comm_errors()
            res[f"finite_{key}"] = bool(torch.isfinite(p).all())
            eng.close()
            return p

        p_fused = train("fused")
        # the split step (4 workgroups per sample) through the exchange (per-rank batch 8: the two
        # ranks share this one GPU, and every split-step workgroup fills a CU -- at batch 32 a
        # rank spinning in its exchange could hold the CUs its peer's training step waits for;
        # one process per GPU has no such contention)
        p_fs = train("fused", "fused_split", split=True, gb=16)
        p_pg = train("rccl", "pg")
        p_pgs = train("rccl", "pg_split", split=True, gb=16)
        # both sum the same rank-local gradients in rank order: bitwise-identical training
        res["fused_equals_pg"] = torch.equal(p_fused, p_pg)
        res["fused_split_equals_pg_split"] = torch.equal(p_fs, p_pgs)
        if not (res["fused_equals_pg"] and res["fused_split_equals_pg_split"]):
            bounds = (("conv1", 0, 260), ("conv2", 260, 5280), ("fc1", 5280, 21330), ("fc2", 21330, 21840))
            for name, (x, y) in (("plain", (p_fused, p_pg)), ("split", (p_fs, p_pgs))):
                d = (x - y).abs()
                res[f"maxdiff_{name}"] = float(d.max())
                res[f"ndiff_{name}"] = {k: int((d[lo:hi] > 0).sum()) for k, lo, hi in bounds}
        q.put((rank, res))
        dist.destroy_process_group()
    except Exception as e:  # report, do not hang the parent
        q.put((rank, {"exception": repr(e)}))


def test_fused_exchange_two_ranks_one_gpu():
    """Two ranks share the box's one GPU: the fused exchange (lenet_update pushes to the peer and
    sums in rank order) trains bitwise like the process group's all-reduce, in graph replays, the
    native executor and eager steps, with the plain and the split step; no wait times out.
    Every comparison is strict in every run (the one-shot IPC kernel, whose shared-GPU runs
    depended on co-scheduling, is no longer a training path: its test is the deterministic
    loopback one in tests/test_exchange_loopback_gpu.py)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(2):
        r, res = q.get(timeout=300)
        results[r] = res
    for p in procs:
        p.join(timeout=60)
    both = "\n".join(f"rank {r}: {results[r]}" for r in range(2))
    for r in range(2):
        assert "exception" not in results[r], both
    for r in range(2):
        res = results[r]
        for mode, kind in (("fused", "fused-ipc"), ("fused_split", "fused-ipc"), ("pg", "rccl"),
                           ("pg_split", "rccl")):
            mine = {k: v for k, v in res.items() if k.endswith("_" + mode)}
            assert res[f"engine_errors_{mode}"] == 0, (r, mode, mine)  # first: explains a mismatch
            assert res[f"kind_{mode}"] == kind, (r, mode, mine)
            assert res[f"params_equal_{mode}"] and res[f"finite_{mode}"], (r, mode, mine)
        assert res["step_fused"] == "two kernels", res
        assert res["native_fused"] and res["native_fused_split"], res
        assert not res["native_pg"], res
        assert res["fused_equals_pg"] and res["fused_split_equals_pg_split"], f"rank {r}: {both}"
        assert res["split_fused_split"] and not res["split_fused"], res


def _tail_worker(rank, world, port, q):
    """Fused exchange with a per-rank batch whose FC work splits K over waves (B = 256) and an
    epoch tail in another split bucket (B = 100): two epochs of graph-replayed steps + tails.
    The exchange tags are per-workgroup call counters, so the workgroup -> exchange-word map
    must not depend on the batch (counters drifting between full and tail steps
    made ranks add a peer's stale gradient, or time out)."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CSED_IPC_TIMEOUT_S="30")
        import torch.distributed as dist

        from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist
        from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer
        from csed_514_project_distributed_training_using_pytorch_amd.models import Net
        from csed_514_project_distributed_training_using_pytorch_amd.parallel.comm import DistContext
        from csed_514_project_distributed_training_using_pytorch_amd.parallel.sampler import ShardSampler

        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        ctx = DistContext(rank, world, 0, dev, "gloo")
        n = 2 * (2 * 256 + 100)  # per rank: 2 full steps of 256 + a tail of 100
        data = synthetic_mnist(n, seed=5)
        res = {}
        finals = {}
        # reference: the process group's all-reduce (gloo here: host sum, eager steps), bitwise
        # the same rank-ordered sum as the fused exchange
        for mode in ("fused", "rccl"):
            os.environ["CSED_ALLREDUCE"] = mode
            torch.manual_seed(1)
            eng = FusedLeNetTrainer(Net().to(dev), data, lr=0.05, global_batch=512, ctx=ctx)
            smp = ShardSampler(n, world, rank, shuffle=True, seed=42)
            for epoch in range(2):
                smp.set_epoch(epoch)
                eng.train_epoch(smp.indices(), steps_per_graph=2)
            torch.cuda.synchronize(dev)
            p = eng.flat.data.cpu()
            other = p.clone()
            dist.broadcast(other, src=0)
            res[f"kind_{mode}"] = eng.allreduce_kind
            res[f"equal_{mode}"] = torch.equal(p, other)
            res[f"errors_{mode}"] = eng.comm_errors()
            res[f"tail_{mode}"] = eng.tail_size()
            finals[mode] = p
            eng.close()
        res["fused_equals_pg"] = torch.equal(finals["fused"], finals["rccl"])
        q.put((rank, res))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, {"exception": repr(e)}))


def test_fused_exchange_large_batch_with_tail_two_ranks():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tail_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(2):
        r, res = q.get(timeout=300)
        results[r] = res
    for p in procs:
        p.join(timeout=60)
    for r in range(2):
        res = results[r]
        assert "exception" not in res, res
        assert res["errors_fused"] == 0 and res["errors_rccl"] == 0, res
        assert res["kind_fused"] == "fused-ipc" and res["kind_rccl"] == "rccl", res
        assert res["tail_fused"] == 100, res
        assert res["equal_fused"] and res["equal_rccl"] and res["fused_equals_pg"], res


def _rccl_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CSED_ALLREDUCE="rccl")
        import torch.distributed as dist

        from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist
        from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer
        from csed_514_project_distributed_training_using_pytorch_amd.models import Net
        from csed_514_project_distributed_training_using_pytorch_amd.parallel.comm import init_distributed
        from csed_514_project_distributed_training_using_pytorch_amd.parallel.sampler import ShardSampler

        ctx = init_distributed(rank=rank, world_size=world, local_rank=rank, backend="nccl", device="cuda")
        data = synthetic_mnist(2048, seed=3)
        torch.manual_seed(1)
        eng = FusedLeNetTrainer(Net().to(ctx.device), data, lr=0.05, global_batch=64, ctx=ctx)
        smp = ShardSampler(2048, world, rank, shuffle=True, seed=42)
        smp.set_epoch(0)
        eng.set_epoch_order(smp.indices())
        eng.run_steps(12, steps_per_graph=4)
        torch.cuda.synchronize(ctx.device)
        p = eng.flat.data.clone()
        other = p.clone()
        dist.broadcast(other, src=0)
        q.put((rank, {"kind": eng.allreduce_kind, "captured": eng.capture_comm_ok, "equal": torch.equal(p, other),
                      "finite": bool(torch.isfinite(p).all())}))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, {"exception": repr(e)}))


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (one rank per GPU on RCCL)")
def test_rccl_fallback_captured_two_gpus():
    """CSED_ALLREDUCE=rccl on a 2-rank RCCL process group, one rank per GPU: the step
    (reduce-only update -> RCCL all-reduce -> SGD kernel) is captured in a HIP graph and
    both replicas end bitwise identical."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rccl_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    for r in range(2):
        res = results[r]
        assert "exception" not in res, res
        assert res["kind"] == "rccl" and res["captured"] is True, res
        assert res["equal"] and res["finite"], res
