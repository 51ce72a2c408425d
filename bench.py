#!/usr/bin/env python3
"""Headline benchmark: MNIST `Net` data-parallel training throughput on MI355X.

Metric (BASELINE.json): "MNIST epoch time (s) + images/sec at 1/2/4/8 MI355X (DDP)".
Config: the reference's DDP config -- global batch 64 split over N ranks
(strong scaling, ref src/train_dist.py:124,133), SGD lr 0.02 momentum 0.5,
Dropout2d + dropout active, 60,000 synthetic 1x28x28 uint8 images (no network
here, so no real MNIST) sharded with DistributedSampler(seed=42) index math,
random-init weights (torch.manual_seed(1)), bf16 MFMA compute (or fp16 / fp32)
with fp32 master weights / optimizer.

Usage:
    python bench.py [--gpus N] [--steps K] [--warmup W]          # N > 1: spawns N ranks itself
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Order of work on every rank (one process per GPU, RCCL process group for N > 1):

1. setup: process group, synthetic data, engine, HIP-graph capture of every step
   graph the run will replay (capture is never inside a timed region);
2. epoch 0, the reference's own quantity: all 938 steps (incl. the short last
   batch) + the 10k-image validation pass.  ``time_elapsed_s`` = the reference's
   span: t0 taken right after ``import torch`` and the package imports (ref
   src/train_dist.py:1-11 imports, :119 t0), to the end of epoch-0 validation
   (:112 print); everything the reference does after its t0 (rendezvous, data set,
   model) is inside it, and no job work starts before it.  ``process_elapsed_s``
   = process start -> the same point (imports included); ``epoch0_s`` = the
   epoch itself;
3. W warm-up steps, then one untimed rehearsal of exactly the graph sequence
   the timed region replays (so every graph it uses has been replayed before);
4. exactly K timed steps (each = full forward, backward, gradient all-reduce for
   N > 1, SGD update) from the start of an epoch, bracketed by barrier + device
   synchronisation; the time reported is the max over ranks -> ``value`` =
   whole-job images/s, ``ms_per_step``;
5. ``epoch_s``: one more full epoch + validation, warm (steady-state epoch time);
6. N > 1: a bitwise replica check of the parameters and momentum over all ranks
   (``replicas_identical``); a run whose replicas differ reports no value;
7. unless the run itself is fp32 (or ``--no-fp32-record``): the same K-step
   window and warm epoch again on the exact-fp32 kernels, the reference's own
   precision, as the ``fp32`` sub-record.

Rank 0 prints one JSON line.
"""
from __future__ import annotations

import time

T_PROC = time.time()  # process start (process_elapsed_s); the reference's t0 comes after the imports

import argparse  # noqa: E402
import json  # noqa: E402
import os  # noqa: E402
import sys  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# reference epoch times, converted to images/s: 60000 / t
BASELINE_EPOCH_S = {1: 17.53, 2: 11.29, 4: 7.60, 8: 5.00}
METRIC = "MNIST epoch time (s) + images/sec at 1/2/4/8 MI355X (DDP)"


def parse(argv=None) -> argparse.Namespace:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--global-batch", type=int, default=64)
    ap.add_argument("--dtype", choices=["bf16", "fp16", "fp32"], default="bf16")
    ap.add_argument("--steps-per-graph", type=int, default=32)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-epoch", action="store_true", help="skip the warm measured epoch (step 5)")
    ap.add_argument("--grid", type=int, default=0, help="workgroups per step (0 = per-rank batch, max 256)")
    ap.add_argument("--backend", choices=["auto", "nccl", "gloo"], default="auto",
                    help="process group: auto = RCCL ('nccl') on GPUs; gloo lets ranks share one GPU "
                         "(rehearsal of the multi-rank path; the gradient exchange still runs on the GPU)")
    ap.add_argument("--loopback-world", type=int, default=0, metavar="N",
                    help="one GPU only: run lenet_update's fused exchange with N-1 virtual peers (slots of "
                         "this rank's own buffer) -- the per-rank step of an N-GPU run minus the xGMI flight "
                         "time; use with --global-batch 64/N")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: plumbing only (launch/rendezvous/JSON contract), stock PyTorch ops")
    ap.add_argument("--no-fp32-record", action="store_true",
                    help="skip the exact-fp32 sub-record (step 7) of a 16-bit run")
    ap.add_argument("--eager-rccl", action="store_true",
                    help="N > 1: create the RCCL communicator at init_process_group (inside the reference span) "
                         "instead of at its first collective; the bring-up's host collectives then run on it too")
    ap.add_argument("--epoch0-stamps", action="store_true",
                    help="keep every launch's GPU / host time of epoch 0 and the warm epoch in the JSON "
                         "(epoch0_breakdown.replay_gpu_ms); the summary is always there")
    ap.add_argument("--inject-exchange-fault", action="store_true",
                    help="fault-injection test hook: the last rank's exchange pushes go to a dead-end buffer "
                         "(in loopback mode: every virtual peer is dead), so peer waits time out; the bench "
                         "must detect it and re-measure on the process-group all-reduce (config.comm_retry)")
    return ap.parse_args(argv)


def reduce_max(ctx, values: dict) -> dict:
    """{name: seconds} -> the max over ranks of each entry (one collective)."""
    import torch
    import torch.distributed as dist

    from csed_514_project_distributed_training_using_pytorch_amd.parallel.comm import ctl_all_reduce, ctl_device

    if not ctx.is_distributed or not values:
        return dict(values)
    keys = sorted(values)
    t = torch.tensor([float(values[k]) for k in keys], dtype=torch.float64, device=ctl_device(ctx))
    ctl_all_reduce(ctx, t, dist.ReduceOp.MAX)
    return dict(zip(keys, t.tolist()))


def spawn(args: argparse.Namespace, argv: list[str]) -> int:
    """--gpus N > 1 without a torchrun environment: start N ranks (one per GPU) as child
    processes and return the first failing exit code.  Nothing here touches the GPU (the
    launcher module is loaded on its own, without the package), so the children own it."""
    import importlib.util

    spec = importlib.util.spec_from_file_location(
        "_csed_launch", os.path.join(ROOT, "csed_514_project_distributed_training_using_pytorch_amd", "parallel",
                                     "launch.py"))
    launch = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(launch)
    return launch.launch(args.gpus, [sys.executable, os.path.abspath(__file__), *argv],
                         env_extra={"CSED_BENCH_PROC_T0": repr(T_PROC)})


def epoch_chunks(k: int, pos: int, full: int) -> list[int]:
    """How ``advance(k)`` splits k steps from epoch position pos at epoch boundaries."""
    out = []
    while k > 0:
        if pos >= full:
            pos = 0
        n = min(k, full - pos)
        out.append(n)
        pos += n
        k -= n
    return out


def run_cpu(args, ctx, t_start: float, t_proc: float) -> dict:
    """CPU plumbing run (no GPU on this machine): the same launch / rendezvous / timing /
    JSON contract on stock PyTorch ops through the modular trainer.  Not a performance
    number: the JSON says so in ``config.engine``."""
    import torch

    from csed_514_project_distributed_training_using_pytorch_amd.data import DeviceLoader, synthetic_mnist
    from csed_514_project_distributed_training_using_pytorch_amd.engine.modular import ModularTrainer
    from csed_514_project_distributed_training_using_pytorch_amd.models import Net
    from csed_514_project_distributed_training_using_pytorch_amd.parallel.comm import (all_reduce_max, barrier,
                                                                                     replica_checksum)
    from csed_514_project_distributed_training_using_pytorch_amd.parallel.sampler import ShardSampler

    n = ctx.world_size
    train = synthetic_mnist(max(args.global_batch * (args.steps + args.warmup) // 1, args.global_batch), seed=0)
    torch.manual_seed(1)
    tr = ModularTrainer(Net(), lr=0.02, momentum=0.5, ctx=ctx, loss="ce")
    sampler = ShardSampler(len(train), n, ctx.rank, shuffle=True, seed=42)
    loader = DeviceLoader(train, args.global_batch // n, sampler=sampler, device=ctx.device)
    it = iter(loader)
    for _ in range(args.warmup):
        tr.train_batch(*next(it))
    barrier(ctx)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.train_batch(*next(it))
    barrier(ctx)
    elapsed = all_reduce_max(ctx, time.perf_counter() - t0)
    now = time.time()
    same, _, _ = replica_checksum(ctx, torch.cat([p.detach().reshape(-1) for p in tr.model.parameters()]))
    return {"elapsed": elapsed, "engine": "CPU plumbing (stock PyTorch ops, modular trainer): not a GPU number",
            "allreduce": f"process group ({ctx.backend})" if ctx.is_distributed else "none",
            "time_elapsed_s": all_reduce_max(ctx, now - t_start), "process_elapsed_s": all_reduce_max(ctx, now - t_proc),
            "replicas": same}


def start_native_data():
    """The data set, generated natively (csrc/data/synth_mnist.cpp) in a background thread
    that runs while ``import torch`` does: this file loads data/native_synth.py by path (numpy +
    ctypes, not the package, which imports torch).  None when the library is not built."""
    import importlib.util

    path = os.path.join(ROOT, "csed_514_project_distributed_training_using_pytorch_amd", "data", "native_synth.py")
    spec = importlib.util.spec_from_file_location("_csed_native_synth", path)
    ns = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ns)
    if not ns.available():
        return None
    return ns.Job(60000, 10000, seed=0)


def start_gpu_context(phases: dict | None = None, torch_too: bool = True, preload_mask: int = 0):
    """This rank's HIP context, created in a thread started at t0 that runs while the data set
    is generated and the process group comes up.  ctypes loads the HIP runtime that torch
    itself links (torch/lib/libamdhip64.so), so torch later finds this process's primary
    context already up.  The thread's own wall time goes to ``phases["hip_ctx_thread"]``.
    None when there is no such library (CPU-only torch) or no GPU."""
    import ctypes
    import importlib.util
    import threading

    try:
        spec = importlib.util.find_spec("torch")
        lib = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
        if not os.path.exists(lib):
            return None
        hip = ctypes.CDLL(lib)
    except Exception:  # (no torch / no ROCm build: torch brings the context up itself)
        return None
    dev = int(os.environ.get("LOCAL_RANK", "0"))

    def preload(d):
        t = time.time()
        try:
            import torch

            from csed_514_project_distributed_training_using_pytorch_amd.ops import _native

            if _native.load(build_if_missing=False):
                torch.ops.csed.preload_kernels(d, preload_mask)
        except Exception as e:  # (diagnostic only: the kernels then load at their first launch)
            print(f"[bench] kernel preload failed: {e!r}", file=sys.stderr)
        if phases is not None:
            phases["preload_thread"] = time.time() - t

    def run():
        t = time.time()
        sub = {}
        n = ctypes.c_int(0)
        if hip.hipGetDeviceCount(ctypes.byref(n)) != 0 or n.value <= 0:
            return
        sub["ctx.device_count"] = time.time() - t
        if hip.hipSetDevice(dev % n.value) == 0:
            t1 = time.time()
            hip.hipFree(ctypes.c_void_p(0))  # (the context's creation)
            sub["ctx.hip_context"] = time.time() - t1
            if preload_mask:
                # the kernels' code objects load in a thread of their own, beside torch's CUDA
                # set-up below and the engine's: the HIP runtime would otherwise load each
                # translation unit's at its first launch (lenet_tile's: the epoch-0 validation,
                # 5-60 ms on a fresh box, profiles/r6/epoch0.md)
                threading.Thread(target=preload, args=(dev % n.value,), name="csed-preload", daemon=True).start()
            if torch_too:
                # torch's own CUDA state (lazy init, caching allocator: ~0.09 s, round-5 bring-up
                # breakdown engine.net) comes up here too, behind the data generator
                import torch

                t1 = time.time()
                torch.cuda.set_device(dev % n.value)
                sub["ctx.torch_init"] = time.time() - t1
                # (the process's first pageable host -> device copy sets up the runtime's staging
                # buffers: 0.09 s, measured as engine.net in round 5 -- done here, off the path)
                t1 = time.time()
                torch.empty(1, device=torch.device("cuda", dev % n.value)).copy_(torch.zeros(1))
                sub["ctx.first_copy"] = time.time() - t1
        if phases is not None:
            phases.update(sub)
            phases["hip_ctx_thread"] = time.time() - t

    t = threading.Thread(target=run, name="csed-hip-context", daemon=True)
    t.start()
    return t


class EpochStamps:
    """HIP events + host clock at each launch boundary of one epoch (graph replays, the tail step,
    the validation pass).  Recording an event is one small packet per replay (30 per epoch), so
    epoch 0 is always stamped: its breakdown shows where a cold epoch loses time against a warm one
    (a slow first replay: graph upload / first launch; slow early replays that speed up: GPU clock
    ramp; a slow validation: first launch of the eval kernel)."""

    def __init__(self, device):
        import torch

        self.torch = torch
        self.device = device
        self.marks: list[tuple[str, object, float]] = []

    def mark(self, name: str) -> None:
        ev = self.torch.cuda.Event(enable_timing=True)
        ev.record(self.torch.cuda.current_stream(self.device))
        self.marks.append((name, ev, time.perf_counter()))

    def summary(self, detail: bool = False) -> dict | None:
        if len(self.marks) < 2:
            return None
        self.marks[-1][1].synchronize()
        gpu = [a[1].elapsed_time(b[1]) for a, b in zip(self.marks, self.marks[1:])]
        host = [1e3 * (b[2] - a[2]) for a, b in zip(self.marks, self.marks[1:])]
        names = [b[0] for b in self.marks[1:]]
        rep = [g for g, n in zip(gpu, names) if n == "replay"]
        rh = [h for h, n in zip(host, names) if n == "replay"]
        srt = sorted(rep[1:]) if len(rep) > 1 else rep
        med = srt[len(srt) // 2] if srt else None
        r = lambda v: round(v, 4) if v is not None else None  # noqa: E731
        out = {"replays": len(rep), "replay_gpu_ms_total": r(sum(rep)), "first_replay_gpu_ms": r(rep[0]) if rep else None,
               "replay_gpu_ms_median_after_first": r(med), "replay_gpu_ms_last": r(rep[-1]) if rep else None,
               "replays_over_1p2x_median": sum(1 for g in rep if med and g > 1.2 * med),
               "first_replay_host_ms": r(rh[0]) if rh else None, "replay_host_ms_total": r(sum(rh)),
               "tail_gpu_ms": r(sum(g for g, n in zip(gpu, names) if n == "tail")),
               "eval_gpu_ms": r(sum(g for g, n in zip(gpu, names) if n == "eval")),
               "eval_host_ms": r(sum(h for h, n in zip(host, names) if n == "eval")),
               "gpu_ms_total": r(sum(gpu)), "host_ms_total": r(sum(host))}
        if detail:
            out["replay_gpu_ms"] = [r(g) for g in rep]
            out["replay_host_ms"] = [r(h) for h in rh]
        return out


# the order of bring-up events on this rank, for tests/test_bench_contract_cpu.py: (name, time)
BRINGUP_EVENTS: list[tuple[str, float]] = []


def bringup(args, phases: dict):
    """Imports, then the reference's t0, then the job's first work (ref src/train_dist.py:1-11
    imports torch / torchvision / matplotlib / tqdm, :119 takes t0, :146 rendezvous, :148 data):
    ``import torch`` and the package are timed apart (``import_torch``, ``import_pkg``) and
    fall outside ``time_elapsed_s``; the synthetic-data generator and the HIP-context thread
    start only after t0.  Returns (t0, native data job, HIP-context thread)."""
    t_mark = time.time()
    import torch  # noqa: F401
    phases["import_torch"] = time.time() - t_mark
    t_mark = time.time()
    import torch.distributed  # noqa: F401

    import csed_514_project_distributed_training_using_pytorch_amd.parallel.comm  # noqa: F401
    import csed_514_project_distributed_training_using_pytorch_amd.utils.prof  # noqa: F401
    if args.device == "cuda":
        import csed_514_project_distributed_training_using_pytorch_amd.engine.fused  # noqa: F401
    phases["import_pkg"] = time.time() - t_mark
    t_start = time.time()  # the reference's t0 (src/train_dist.py:119)
    BRINGUP_EVENTS.append(("t0", t_start))
    native_job = ctx_job = None
    if args.device == "cuda" and not os.environ.get("CSED_TORCH_DATA"):
        BRINGUP_EVENTS.append(("native_data", time.time()))
        native_job = start_native_data()
    if args.device == "cuda":
        BRINGUP_EVENTS.append(("hip_ctx_thread", time.time()))
        # code objects: lenet_fused (the step), lenet_tile (the 10k validation, and large batches),
        # lenet_fused_f32 (--dtype fp32 and the fp32 sub-record), the exchange (N > 1)
        # (CSED_PRELOAD=1: a third thread loads them beside the context's creation -- measured, it
        # only contends with it: profiles/r6/epoch0.md; by default each loads at its first launch)
        ctx_job = start_gpu_context(phases, preload_mask=0b1111 if os.environ.get("CSED_PRELOAD") == "1" else 0)
    return t_start, native_job, ctx_job


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn(args, argv)
    t_proc = float(os.environ.get("CSED_BENCH_PROC_T0", T_PROC))
    # bring-up phases (s) on this rank; the JSON reports the max over ranks of each
    phases = {"spawn": T_PROC - t_proc}
    t_start, native_job, ctx_job = bringup(args, phases)
    import torch
    import torch.distributed as dist

    from csed_514_project_distributed_training_using_pytorch_amd.parallel.comm import (
        all_reduce_max, barrier, init_distributed, rendezvous, replica_checksum)
    from csed_514_project_distributed_training_using_pytorch_amd.utils import prof

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        return 2
    backend = None if args.backend == "auto" else args.backend
    data_job = None
    if args.device == "cuda" and native_job is None:  # the data set builds (CPU threads) while the GPU context comes up
        from concurrent.futures import ThreadPoolExecutor

        from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist

        pool = ThreadPoolExecutor(1)
        data_job = pool.submit(lambda: (synthetic_mnist(60000, seed=0, train=True),
                                        synthetic_mnist(10000, seed=0, train=False)))
        pool.shutdown(wait=False)
    t_mark = time.time()
    # N > 1: the rendezvous (waiting for every rank to connect: their imports end at different
    # times) runs here, in the main thread, while this rank's HIP context comes up in its thread;
    # the process group (RCCL communicator) is then built on the same store
    store = rendezvous(world_size=world) if world > 1 else None
    phases["rendezvous"] = time.time() - t_mark
    # RCCL's communicator is created lazily (at its first collective: the fallback all-reduce, or
    # the fused-vs-RCCL path timing after epoch 0) with a gloo control plane for the bring-up's
    # host collectives: creating it takes 1.0-3.6 s even for one rank (tools/rccl_init_probe.py),
    # and the fused step's gradients travel over the in-kernel IPC exchange.  Such a process
    # group touches no GPU: it comes up here too, beside the HIP-context thread
    lazy = args.device == "cuda" and world > 1 and backend in (None, "nccl") and not args.eager_rccl
    ctx = None
    if lazy:
        ctx = init_distributed(world_size=world, device=args.device, backend=backend, store=store, lazy_rccl=True,
                               set_device=False)
    phases["process_group_init"] = time.time() - t_mark
    if ctx_job is not None:
        ctx_job.join()
    if ctx is None:
        ctx = init_distributed(world_size=world, device=args.device, backend=backend, store=store)
    elif ctx.device.type == "cuda":
        torch.cuda.set_device(ctx.device)
    phases["process_group"] = time.time() - t_mark
    if args.device == "cuda" and os.environ.get("CSED_BENCH_STREAM") == "1":
        # every launch of this rank on one created stream instead of the null stream (A/B knob)
        t_mark = time.time()
        torch.cuda.set_stream(torch.cuda.Stream(ctx.device))
        phases["work_stream"] = time.time() - t_mark
    n = ctx.world_size
    if ctx.is_distributed and dist.get_world_size() != args.gpus:
        raise SystemExit(f"process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")

    if args.device == "cpu":
        r = run_cpu(args, ctx, t_start, t_proc)
        elapsed, extra = r["elapsed"], {}
        cfg_engine, allreduce, step_kind, hip_graph = r["engine"], r["allreduce"], "eager", False
        time_elapsed, epoch0_s, epoch_s, val, loss_avg, comm_err, comm_retry = r["time_elapsed_s"], None, None, \
            None, None, 0, None
        process_elapsed, replicas, fp32_rec = r["process_elapsed_s"], r["replicas"], None
        data_src = e0_rec = ew_rec = None
        from csed_514_project_distributed_training_using_pytorch_amd.parallel import ipc as _ipc_cpu

        xdiag = _ipc_cpu.gather_diag(ctx, dict(_ipc_cpu.empty_diag(ctx), allreduce=r["allreduce"],
                                               note="CPU plumbing run: no exchange")) if n > 1 else None
    else:
        from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer
        from csed_514_project_distributed_training_using_pytorch_amd.models import Net
        from csed_514_project_distributed_training_using_pytorch_amd.parallel.sampler import ShardSampler

        dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[args.dtype]
        t_mark = time.time()
        with prof.range("bench:data"):
            if native_job is not None:
                from csed_514_project_distributed_training_using_pytorch_amd.data.mnist import MNISTData

                (xi, xl), (ti, tl) = native_job.result()
                phases["data_gen_thread"] = native_job.elapsed_s
                train = MNISTData(torch.from_numpy(xi), torch.from_numpy(xl), synthetic=True)
                test = MNISTData(torch.from_numpy(ti), torch.from_numpy(tl), synthetic=True)
                data_src = "native generator (csrc/data/synth_mnist.cpp), overlapped with import torch"
            else:
                train, test = data_job.result()
                data_src = "data/mnist.py:synthetic_mnist (torch CPU ops)"
        phases["data_wait"] = time.time() - t_mark
        use_graph = not args.no_graph

        def sync_barrier():
            torch.cuda.synchronize(ctx.device)
            if ctx.is_distributed:  # (one rank: the barrier is empty, one synchronize suffices)
                barrier(ctx)
                torch.cuda.synchronize(ctx.device)

        def run_once(loopback_world: int, inject: bool, ph: dict, dt=dt, reuse=None):
            t_mark = time.time()
            torch.manual_seed(1)
            net = Net()
            ph["engine.net_cpu"] = time.time() - t_mark
            net = net.to(ctx.device)
            ph["engine.net"] = time.time() - t_mark
            eng = FusedLeNetTrainer(net, train, lr=0.02, momentum=0.5, global_batch=args.global_batch, ctx=ctx,
                                    compute_dtype=dt, grid=args.grid or None, loopback_world=loopback_world,
                                    reuse_exchange=reuse)
            ph["engine"] = time.time() - t_mark
            ph.update({f"engine.{k}": v for k, v in eng.bringup_s.items()})
            if inject and eng.exch is not None and (loopback_world or ctx.rank == ctx.world_size - 1):
                eng.inject_exchange_fault()
            sampler = ShardSampler(len(train), ctx.world_size, ctx.rank, shuffle=True, seed=42)
            state = {"epoch": 0, "pos": 0}
            spg = args.steps_per_graph

            def new_epoch(order=None):
                if order is None:
                    sampler.set_epoch(state["epoch"])
                    order = sampler.indices()
                eng.set_epoch_order(order)
                state["epoch"] += 1
                state["pos"] = 0

            def advance(k: int):
                for n_ in epoch_chunks(k, state["pos"], eng.full_steps()):
                    if state["pos"] >= eng.full_steps():
                        new_epoch()
                    eng.run_steps(n_, spg, use_graph=use_graph)
                    state["pos"] += n_

            def full_epoch(stamps: EpochStamps | None = None):
                plan = eng.step_plan(eng.full_steps(), spg, use_graph)
                if stamps is not None:
                    stamps.mark("start")
                for launch in plan:
                    launch()
                    if stamps is not None:
                        stamps.mark("replay")
                eng.last_partial_step(use_graph=use_graph)
                if stamps is not None:
                    stamps.mark("tail")
                res = eng.evaluate(test)
                if stamps is not None:
                    stamps.mark("eval")
                return res

            new_epoch()
            full = eng.full_steps()
            t_mark = time.time()
            if use_graph:  # the graphs epoch 0 replays (the timed K-step graph: after the span)
                with prof.range("bench:capture"):
                    eng.prepare(spg, ks=(full,))
            ph["capture"] = time.time() - t_mark
            ph.update({k: v for k, v in eng.bringup_s.items() if k.startswith("capture.")})
            t_mark = time.time()
            eng._device_data(test)  # test set upload is data loading (ref: DataLoader), not epoch work
            ph["test_upload"] = time.time() - t_mark
            # 2. epoch 0, cold: the reference's time_elapsed (process start -> epoch-0 validation),
            # every launch stamped (HIP events + host clock; --epoch0-stamps keeps the per-replay list)
            sync_barrier()
            st0 = EpochStamps(ctx.device)
            te = time.perf_counter()
            with prof.range("bench:epoch0"):
                full_epoch(st0)
            sync_barrier()
            ph["epoch0"] = time.perf_counter() - te
            epoch0 = all_reduce_max(ctx, ph["epoch0"])
            now = time.time()
            t_el = all_reduce_max(ctx, now - t_start)  # the reference's span (t0 after the imports)
            p_el = all_reduce_max(ctx, now - t_proc)  # from process start
            # a path timing deferred by the lazy-RCCL bring-up (fused exchange vs RCCL all-reduce;
            # collective, creates the RCCL communicator): outside the span, before anything timed
            t_mark = time.time()
            try:
                switched = eng.select_path()
            except Exception as e:  # (e.g. the RCCL communicator could not be created: the fused
                # exchange, self-tested on every rank, stays; the JSON says why)
                print(f"[bench] path selection failed ({e!r}); keeping {eng.allreduce_kind}", file=sys.stderr)
                eng.exchange_note = f"{eng.exchange_note}; path timing failed: {type(e).__name__}: {e}"
                switched = False
            ph["path_select"] = time.time() - t_mark
            if use_graph:  # the timed window's graphs (outside the span: not epoch-0 work)
                t_mark = time.time()
                eng.prepare(spg, ks=(full, *epoch_chunks(args.steps, 0, full)) if switched
                            else tuple(epoch_chunks(args.steps, 0, full)), tail=switched)
                ph["capture_timed"] = time.time() - t_mark
            # 3. warm-up, then a rehearsal of the timed sequence (same graphs, same order)
            with prof.range("bench:warmup"):
                new_epoch()
                advance(args.warmup)
                new_epoch()
                advance(args.steps)
            sync_barrier()
            eng.take_loss()  # the reported loss covers the timed steps only
            # 4. K timed steps from an epoch start (within one epoch -- the usual case -- the
            # launch plan is resolved before the clock starts: the region holds the launches)
            new_epoch()
            plan = eng.step_plan(args.steps, spg, use_graph) if args.steps <= full else None
            sync_barrier()
            ev = prof.EventTimer(ctx.device).start()
            with prof.range("bench:timed"):  # (the marker push stays outside the clock)
                t0 = time.perf_counter()
                if plan is not None:
                    for launch in plan:
                        launch()
                    state["pos"] += args.steps
                else:
                    advance(args.steps)
                ev.stop()
                sync_barrier()
                t1 = time.perf_counter()
            elapsed = all_reduce_max(ctx, t1 - t0)
            dev_ms = all_reduce_max(ctx, ev.ms())
            loss_sum, _ = eng.take_loss()
            # 5. one more full epoch + validation, warm (order prepared before the clock starts)
            epoch_s = val = stw = None
            if not args.no_epoch:
                sampler.set_epoch(state["epoch"])
                order = sampler.indices()
                new_epoch(order)
                sync_barrier()
                stw = EpochStamps(ctx.device)
                te = time.perf_counter()
                with prof.range("bench:epoch"):
                    vloss, vcorrect = full_epoch(stw)
                sync_barrier()
                epoch_s = all_reduce_max(ctx, time.perf_counter() - te)
                val = {"val_loss": vloss / len(test), "val_acc": vcorrect / len(test)}
            torch.cuda.synchronize(ctx.device)
            # every rank must agree: one rank's timed-out peer wait invalidates the whole run
            err = int(all_reduce_max(ctx, float(eng.comm_errors())))
            # bitwise replica check: a silently wrong exchange cannot pass as a result
            same_p, _, _ = replica_checksum(ctx, eng.flat.data)
            same_m, _, _ = replica_checksum(ctx, eng.momentum_buf)
            return dict(eng=eng, elapsed=elapsed, dev_ms=dev_ms, loss_sum=loss_sum, epoch0=epoch0, t_el=t_el,
                        p_el=p_el,
                        epoch_s=epoch_s, val=val, err=err, replicas=same_p and same_m,
                        e0=st0.summary(args.epoch0_stamps), ew=stw.summary(args.epoch0_stamps) if stw else None,
                        xdiag=eng.exchange_diag(),
                        diag=eng.comm_diag() if err else None)

        from csed_514_project_distributed_training_using_pytorch_amd.parallel import ipc as _ipc

        r = run_once(args.loopback_world, args.inject_exchange_fault, phases)
        comm_retry = None
        first_fault = None
        if ((r["err"] or not r["replicas"]) and r["eng"].exch is not None
                and os.environ.get("CSED_ALLREDUCE", "auto").lower() != "rccl"):
            # a peer wait of the IPC exchange timed out somewhere (or a replica differs): release
            # the IPC buffers on every rank (collective) and measure again on the process group's
            # all-reduce (RCCL on GPUs; loopback mode: the plain one-GPU step), so the reported
            # number is a valid training run
            comm_retry = r["eng"].allreduce_kind
            first_fault = {"error_word": r["err"], "replicas_identical": r["replicas"], "first_mismatch": r["diag"]}
            first_fault_diag = _ipc.gather_diag(ctx, r["xdiag"])
            r["eng"].close()
            del r
            import gc
            gc.collect()
            sync_barrier()
            _ipc.LAST_TIMING = None
            os.environ["CSED_ALLREDUCE"] = "rccl"
            retry_phases = {}
            r = run_once(0, False, retry_phases)
            phases.update({f"retry.{k}": v for k, v in retry_phases.items()})
        eng = r["eng"]
        e0_rec, ew_rec = r["e0"], r["ew"]
        # every rank's exchange diagnostics (collective): peer access, IPC open, self-test, path
        # timing, error word, first mismatch -- names the failing stage of an N-GPU bring-up
        xdiag = _ipc.gather_diag(ctx, r["xdiag"]) if n > 1 else None
        if first_fault is not None:
            first_fault["exchange_diag_first_run"] = first_fault_diag
        elapsed, time_elapsed, epoch0_s, epoch_s, val = r["elapsed"], r["t_el"], r["epoch0"], r["epoch_s"], r["val"]
        process_elapsed = r["p_el"]
        comm_err, replicas = r["err"], r["replicas"]
        loss_avg = r["loss_sum"] / max(1, args.steps * eng.B)
        engine_kernels = {"fused-ipc": " with in-kernel xGMI gradient exchange", "none": ""}.get(
            eng.allreduce_kind, " + gradient all-reduce")
        if eng.loopback_world:
            engine_kernels = f" with the in-kernel exchange looped back to {eng.loopback_world} virtual ranks"
            # the loopback invariant check runs in kernels of its own (CSED_LOOPBACK_CHECK=0: the
            # real world-N update kernel, as tools/exchange_loopback.py times it)
            extra_lb = {"loopback_world": eng.loopback_world,
                        "loopback_check": os.environ.get("CSED_LOOPBACK_CHECK", "1") != "0"}
        else:
            extra_lb = {}
        cfg_engine = f"fused HIP ({eng.kernel_names}{engine_kernels})"
        allreduce, step_kind = eng.allreduce_kind, eng.step_kind
        hip_graph = use_graph and bool(eng.capture_comm_ok)
        extra = {"device_ms_per_step": round(r["dev_ms"] / args.steps, 5), **extra_lb}
        if _ipc.LAST_TIMING:
            extra["allreduce_select_us"] = _ipc.LAST_TIMING
        if eng.path_timing_us:
            extra["step_path_select_us"] = eng.path_timing_us
        if eng.exchange_note:
            extra["exchange"] = eng.exchange_note
        if _ipc.LAST_NOTE:
            extra["allreduce_note"] = _ipc.LAST_NOTE
        if first_fault:
            extra["first_run_fault"] = first_fault
        # 7. the reference's precision (src/model.py: fp32 defaults) on the same window + warm epoch
        fp32_rec = None
        if args.dtype != "fp32" and not args.no_fp32_record and not args.inject_exchange_fault:
            sync_barrier()
            donor = eng if eng.exch is not None and not eng.loopback_world else None
            if donor is None:
                eng.close()
            else:
                donor._graphs.clear()  # (the exchange moves to the fp32 engine: see reuse_exchange)
                donor._stepper = None
            del r, eng
            import gc
            gc.collect()
            sync_barrier()
            f = run_once(args.loopback_world, False, {}, dt=torch.float32, reuse=donor)
            donor = None
            fe = f["eng"]
            fp32_rec = {"ms_per_step": round(1e3 * f["elapsed"] / args.steps, 5),
                        "value": round(args.steps * args.global_batch / f["elapsed"], 1),
                        "device_ms_per_step": round(f["dev_ms"] / args.steps, 5),
                        "epoch_s": round(f["epoch_s"], 4) if f["epoch_s"] is not None else None,
                        "epoch0_s": round(f["epoch0"], 4),
                        "epoch0_breakdown": f["e0"],
                        "engine": f"fused HIP ({fe.kernel_names}), allreduce {fe.allreduce_kind}",
                        "replicas_identical": f["replicas"], "comm_error_word": f["err"]}
            if f["val"]:
                fp32_rec.update({k: round(v, 4) for k, v in f["val"].items()})
            fe.close()

    bringup_rec = {k: round(v, 4) for k, v in reduce_max(ctx, phases).items()}
    value = args.steps * args.global_batch / elapsed
    valid = not comm_err and replicas
    base = BASELINE_EPOCH_S.get(n)
    base_ips = 60000.0 / base if base else None
    if ctx.is_main:
        rec = {
            "metric": METRIC,
            "value": round(value, 1) if valid else None,
            "unit": "images/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 5),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(value / base_ips, 2) if base_ips else None,
            "vs_baseline_basis": "warm-rate: timed-window images/s / the reference's whole-run images/s "
                                 "(like-for-like: vs_baseline_time_elapsed, vs_baseline_epoch)",
            "dtype": args.dtype if args.device == "cuda" else "fp32",
            "data": "synthetic (60000 x 1x28x28 uint8, class-conditional stroke mixture; random-init weights)",
            "data_source": data_src if args.device == "cuda" else "data/mnist.py:synthetic_mnist",
            "config": {"model": "Net (ref src/model.py, 21,840 params)", "global_batch": args.global_batch,
                       "seq_len": None, "parallelism": f"dp{n}", "optimizer": "SGD lr=0.02 momentum=0.5",
                       "engine": cfg_engine, "hip_graph": hip_graph, "allreduce": allreduce, "step": step_kind,
                       "process_group": {"backend": ctx.backend, "ranks": n} if ctx.is_distributed else None,
                       **extra},
            "time_elapsed_s": round(time_elapsed, 4) if time_elapsed is not None else None,
            "process_elapsed_s": round(process_elapsed, 4) if process_elapsed is not None else None,
            "epoch0_s": round(epoch0_s, 4) if epoch0_s is not None else None,
            "epoch_s": round(epoch_s, 4) if epoch_s is not None else None,
            "baseline_epoch_s": base,
            "vs_baseline_time_elapsed": round(base / time_elapsed, 2) if base and time_elapsed else None,
            "vs_baseline_epoch": round(base / epoch_s, 1) if base and epoch_s else None,
            "vs_baseline_note": ("vs_baseline = warm timed-window images/s / the reference's images/s over its "
                                 "whole 1-epoch run (its t0, right after its imports, to the epoch-0 print, incl. "
                                 "rendezvous, data loading and validation); the like-for-like ratios are "
                                 "vs_baseline_time_elapsed (the same span here: t0 after import torch and the "
                                 "package) and vs_baseline_epoch (a warm epoch + validation); process_elapsed_s "
                                 "adds the imports (process start -> the same point)"),
            "replicas_identical": replicas if n > 1 else None,
            "train_loss_timed_rank0": round(loss_avg, 4) if loss_avg is not None else None,
            # where the time goes, max over ranks of each phase (s).  Before t0 (process_elapsed_s
            # only): spawn (launcher -> this process), import_torch, import_pkg.  After t0
            # (time_elapsed_s): process_group (rendezvous, RCCL communicator; includes the wait
            # for the HIP-context thread, hip_ctx_thread = that thread's own time), data_wait
            # (what is left of the native generator), engine (incl. engine.ipc_open /
            # engine.self_test of the fused exchange), capture (HIP graphs), test_upload, epoch0
            # (938 steps + validation)
            "bringup_s": bringup_rec,
            # epoch 0 (inside time_elapsed_s) and the warm epoch, stamped launch by launch (GPU ms
            # between HIP events, host ms between enqueues): where a cold epoch loses time
            "epoch0_breakdown": e0_rec,
            "epoch_breakdown": ew_rec,
            # N > 1: per-rank data-parallel diagnostics (parallel/ipc.py DIAG_KEYS), in rank order
            "exchange_diag": xdiag,
        }
        if comm_retry:
            rec["config"]["comm_retry"] = f"{comm_retry} path timed out; re-measured on the process-group all-reduce"
        if comm_err:
            rec["comm_error"] = (f"IPC exchange error word {comm_err} (1: a peer wait timed out, 2: a received "
                                 "word differed from the value pushed): results invalid")
        if not replicas:
            rec["replica_error"] = "parameters / momentum differ between ranks after the run: results invalid"
        if fp32_rec:
            rec["fp32"] = fp32_rec
            if base and fp32_rec.get("epoch_s"):
                fp32_rec["vs_baseline_epoch"] = round(base / fp32_rec["epoch_s"], 1)
        if val:
            rec.update({k: round(v, 4) for k, v in val.items()})
        print(json.dumps(rec), flush=True)
    if ctx.is_distributed:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
