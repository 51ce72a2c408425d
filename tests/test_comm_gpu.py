"""Native one-shot IPC all-reduce (csrc/comm/ipc_allreduce.hip, parallel/ipc.py) and the
gradient exchange fused into lenet_update (csrc/kernels/lenet_fused.hip, engine/fused.py).

Two ranks share the box's single GPU: the handle exchange, the peer mapping,
the flag protocol (both slot parities, graph replay) and the fused engine's
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


def _oneshot_checks(ar, dist, dev, n, rank) -> dict:
    """The one-shot all-reduce against the process group's reduction: eager calls, then three
    calls per replay of a captured graph (new inputs each replay), then its error word."""
    res = {}
    # random data vs the process group's reduction (2 ranks: a + b in either order)
    g = torch.Generator(device="cpu").manual_seed(100 + rank)
    ok = True
    for _ in range(5):
        x = torch.randn(n, generator=g).to(dev)
        ref = x.cpu().clone()
        dist.all_reduce(ref)
        y = ar(x.clone())
        ok &= torch.equal(y.cpu(), ref)
    res["eager"] = ok
    buf = torch.zeros(n, device=dev)
    out = [torch.zeros(n, device=dev) for _ in range(3)]
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        for k in range(3):
            ar(buf + k, out[k])
    ok = True
    for _ in range(3):
        x = torch.randn(n, generator=g)
        buf.copy_(x.to(dev))
        graph.replay()
        torch.cuda.synchronize(dev)
        for k in range(3):
            ref = (x + k).clone()
            dist.all_reduce(ref)
            ok &= torch.allclose(out[k].cpu(), ref, rtol=0, atol=1e-5)
    res["graph"] = ok
    res["errors"] = ar.error()
    return res


def _worker(rank, world, port, q):
    try:
        # two processes share one GPU here, and how the GPU interleaves their queues is
        # not ours to control: give the peer waits a generous bound (the kernels still
        # report a timeout through the error word, checked below)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CSED_ALLREDUCE="ipc",
                          CSED_IPC_TIMEOUT_S="30")
        import torch.distributed as dist

        from csed_514_project_distributed_training_using_pytorch_amd.parallel.comm import DistContext
        from csed_514_project_distributed_training_using_pytorch_amd.parallel.ipc import make_allreduce

        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        ctx = DistContext(rank, world, 0, dev, "gloo")
        res = {}
        n = 21840
        # The one-shot all-reduce kernel spins until the peer PROCESS's kernel has pushed.  With
        # both processes on this one device, the GPU does not always run the two processes'
        # queues at once: in 3 of 4 runs of one session a 30 s wait ran out somewhere
        # (profiles/dp_exchange_r3.md), sometimes already in make_allreduce's self-test, which
        # then reports the path unusable.  That is a property of two processes sharing a device
        # -- one process per GPU never waits on a co-tenant, and `auto` mode does not pick this
        # path when ranks share a GPU -- so here the one-shot checks are skipped when it is
        # unusable or reported a timed-out wait, and required bitwise otherwise.  The fused
        # exchange (lenet_update), the production path, is checked strictly in every run.
        try:
            ar = make_allreduce(ctx, n)
        except RuntimeError as e:
            if "unusable" not in str(e):
                raise
            ar = None
            res["oneshot_unavailable"] = str(e)
        res["enabled"] = ar is not None
        if ar is not None:
            res.update(_oneshot_checks(ar, dist, dev, n, rank))

        # fused data-parallel engine: identical parameters on both ranks after graph steps
        from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist
        from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer
        from csed_514_project_distributed_training_using_pytorch_amd.models import Net
        from csed_514_project_distributed_training_using_pytorch_amd.parallel.sampler import ShardSampler

        data = synthetic_mnist(2048, seed=3)

        def train(mode, key=None, split=False, gb=64):
            # ipc: reduce-only update -> one-shot IPC all-reduce kernel -> SGD kernel;
            # fused: lenet_update exchanges with the peer itself (one kernel)
            key = key or mode
            os.environ["CSED_ALLREDUCE"] = mode
            torch.manual_seed(1)
            try:
                eng = FusedLeNetTrainer(Net().to(dev), data, lr=0.05, global_batch=gb, ctx=ctx, split=split)
            except RuntimeError as e:  # (collective: every rank raises it)
                if mode != "ipc" or "unusable" not in str(e):
                    raise
                res[f"unavailable_{key}"] = str(e)
                return None
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
            return p

        # The one-shot IPC engine path (reduce-only update -> spinning all-reduce kernel -> SGD
        # kernel; CSED_ALLREDUCE=ipc).  Its pushes are write-through (system-scope) stores
        # (push_word in csrc/comm/ipc_allreduce.hip: plain stores could sit dirty in the writer's
        # L2 while the owner polled memory).  On this shared device it may still be unusable or
        # time out (see above); CSED_TEST_SHARED_GPU_IPC=0 skips it.
        ipc_engine = os.environ.get("CSED_TEST_SHARED_GPU_IPC", "1") == "1"
        p_ipc = train("ipc") if ipc_engine else None
        res["ipc_engine"] = ipc_engine
        p_fused = train("fused")
        # the split step (4 workgroups per sample) through both exchange paths
        # (per-rank batch 8: the two ranks share this one GPU, and every split-step workgroup
        # fills a CU -- at batch 32 (2 x 128 of them) a rank spinning in its exchange could
        # hold the CUs its peer's training step waits for; one process per GPU has no such
        # contention)
        p_fs = train("fused", "fused_split", split=True, gb=16)
        p_is = train("ipc", "ipc_split", split=True, gb=16) if ipc_engine else None
        # both sum the same rank-local gradients in rank order: bitwise-identical training
        # (None: not compared -- the one-shot path was unavailable or a wait timed out on a rank)
        def same(x, y, key):
            err = torch.tensor([float(res.get(f"engine_errors_{key}") or 0)])
            dist.all_reduce(err, op=dist.ReduceOp.MAX)  # (gloo, CPU: every rank runs it)
            return None if x is None or err.item() else torch.equal(x, y)

        res["fused_split_equals_ipc_split"] = same(p_is, p_fs, "ipc_split")
        res["fused_equals_ipc"] = same(p_ipc, p_fused, "ipc")
        bad = torch.tensor([1.0 if (res["fused_equals_ipc"] is False or res["fused_split_equals_ipc_split"] is False)
                            else 0.0])
        dist.all_reduce(bad, op=dist.ReduceOp.MAX)  # (the diagnostics below are collective)
        if bad.item():
            # diagnostics: which path is the outlier (the process group's all-reduce as a third
            # opinion) and which parameters differ
            try:
                p_pg = train("rccl", "pg")
                res["pg_equals_fused"] = torch.equal(p_pg, p_fused)
                res["pg_equals_ipc"] = p_ipc is not None and torch.equal(p_pg, p_ipc)
            except Exception as e:  # (diagnostics only)
                res["pg_error"] = repr(e)
            bounds = (("conv1", 0, 260), ("conv2", 260, 5280), ("fc1", 5280, 21330), ("fc2", 21330, 21840))
            for name, (x, y) in (("ipc", (p_ipc, p_fused)), ("ipc_split", (p_is, p_fs))):
                if x is not None:
                    d = (x - y).abs()
                    res[f"maxdiff_{name}"] = float(d.max())
                    res[f"ndiff_{name}"] = {k: int((d[lo:hi] > 0).sum()) for k, lo, hi in bounds}
        q.put((rank, res))
        dist.destroy_process_group()
    except Exception as e:  # report, do not hang the parent
        q.put((rank, {"exception": repr(e)}))


def test_ipc_allreduce_two_ranks_one_gpu():
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
    # (both ranks' records in full on any failure: one rank's exception usually shows on the
    # other as a reset connection)
    both = "\n".join(f"rank {r}: {results[r]}" for r in range(2))
    for r in range(2):
        assert "exception" not in results[r], both
    # A timed-out wait on EITHER rank voids that mode's comparisons: the rank that gave up sums
    # without its peer, so the replicas differ although the other rank reports nothing
    # (seen: rank 1 clean, rank 0 timed out after a ~30 s co-scheduling stall)
    def timed_out(key):
        return any(results[r].get(key) for r in range(2))

    for r in range(2):
        res = results[r]
        # the one-shot kernel: bitwise right unless unusable here or a wait timed out (see
        # _worker); the error words are checked first, since a timeout explains a mismatch
        if res["enabled"] and not timed_out("errors"):
            assert res["eager"] and res["graph"], res
        modes = (("ipc", "ipc-oneshot"), ("ipc_split", "ipc-oneshot")) if res["ipc_engine"] else ()
        for mode, kind in modes + (("fused", "fused-ipc"), ("fused_split", "fused-ipc")):
            mine = {k: v for k, v in res.items() if k.endswith("_" + mode)}
            if mode.startswith("ipc"):
                if f"unavailable_{mode}" in res:
                    continue
                assert res[f"kind_{mode}"] == kind, (r, mode, mine)
                assert res[f"finite_{mode}"], (r, mode, mine)
                if timed_out(f"engine_errors_{mode}"):
                    continue  # a timed-out wait: partial sums, nothing to compare
            else:  # the fused exchange: strict in every run
                assert res[f"engine_errors_{mode}"] == 0, (r, mode, mine)  # first: explains a mismatch
                assert res[f"kind_{mode}"] == kind, (r, mode, mine)
            assert res[f"params_equal_{mode}"] and res[f"finite_{mode}"], (r, mode, mine)
        assert res["step_fused"] == "two kernels", res
        assert res["native_fused"] and res["native_fused_split"], res
        assert not res.get("native_ipc", False), res
        diag = {k: v for k, v in res.items()
                if k.startswith(("maxdiff", "ndiff", "engine_errors", "errors", "pg_equals", "fused_equals",
                                 "fused_split_equals"))}
        assert res["fused_equals_ipc"] is not False and res["fused_split_equals_ipc_split"] is not False, \
            f"rank {r}: {diag}\n{both}"
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
