"""Data-parallel step time of the fused engine per gradient-exchange path.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/dp_step_bench.py [--gloo]

Paths: ``fused`` (exchange inside lenet_update: 2 kernels per step), ``ipc``
(reduce-only update -> one-shot IPC all-reduce kernel -> SGD kernel) and, on an
RCCL process group, ``rccl`` (same with RCCL's all-reduce).  Each is timed as
graph-replayed steps (engine._time_steps, max over ranks).  With --gloo the
bootstrap group is gloo and the ranks may share one GPU (their kernels then
compete for it, and the transport is local HBM, not xGMI).
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.parallel.comm import DistContext  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.parallel.sampler import ShardSampler  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gloo", action="store_true")
    ap.add_argument("--global-batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--no-time-steps", action="store_true", help="skip engine._time_steps (bench.py's order)")
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    dev = torch.device("cuda", 0 if args.gloo else local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if args.gloo:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ctx = DistContext(rank, world, local, dev, "gloo")
    else:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        ctx = DistContext(rank, world, local, dev, "nccl")
    data = synthetic_mnist(60000, seed=0)
    modes = ["fused"] + ([] if args.gloo else ["rccl"])
    out = {}
    for mode in modes:
        os.environ["CSED_ALLREDUCE"] = mode
        torch.manual_seed(1)
        eng = FusedLeNetTrainer(Net().to(dev), data, lr=0.02, momentum=0.5, global_batch=args.global_batch, ctx=ctx)
        smp = ShardSampler(len(data), world, rank, shuffle=True, seed=42)
        smp.set_epoch(0)
        eng.set_epoch_order(smp.indices())
        us = float("nan") if args.no_time_steps else eng._time_steps(nsteps=args.steps, reps=10)
        # the same steps the way bench.py runs them: cached graphs, wall clock
        eng.prepare(args.steps)
        eng.run_steps(4 * args.steps, args.steps)
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        eng.run_steps(16 * args.steps, args.steps)
        torch.cuda.synchronize(dev)
        wall_us = (time.perf_counter() - t0) * 1e6 / (16 * args.steps)
        out[mode] = (eng.allreduce_kind, round(us, 2), eng.comm_errors(), round(wall_us, 2))
        del eng
        torch.cuda.synchronize(dev)
    if rank == 0:
        for mode, (kind, us, err, wall) in out.items():
            print(f"world={world} backend={ctx.backend} global_batch={args.global_batch} path={mode:5s} "
                  f"kind={kind:11s} step_us={us:7.2f} run_steps_wall_us={wall:7.2f} comm_errors={err}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
