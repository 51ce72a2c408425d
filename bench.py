#!/usr/bin/env python3
"""Headline benchmark: MNIST `Net` data-parallel training throughput on MI355X.

Metric (BASELINE.json): "MNIST epoch time (s) + images/sec at 1/2/4/8 MI355X (DDP)".
Config: the reference's DDP config -- global batch 64 split over N ranks
(strong scaling, ref src/train_dist.py:124,133), SGD lr 0.02 momentum 0.5,
Dropout2d + dropout active, 60,000 synthetic 1x28x28 uint8 images (no network
here, so no real MNIST) sharded with DistributedSampler(seed=42) index math,
random-init weights (torch.manual_seed(1)), bf16 MFMA compute with fp32
master weights / optimizer.

Usage:
    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

W untimed warm-up steps, then exactly K timed steps (each = full forward,
backward, gradient all-reduce over RCCL for N > 1, and SGD update),
bracketed by barrier + device synchronisation; the time reported is the max
over ranks.  Rank 0 prints one JSON line; ``value`` is the whole-job
images/second.  ``epoch_s`` additionally reports a measured full epoch (938
steps incl. the short last batch + the 10k-image validation pass), the
reference's own "time to train 1 epoch" quantity.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# reference epoch times, converted to images/s: 60000 / t
BASELINE_EPOCH_S = {1: 17.53, 2: 11.29, 4: 7.60, 8: 5.00}
METRIC = "MNIST epoch time (s) + images/sec at 1/2/4/8 MI355X (DDP)"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--global-batch", type=int, default=64)
    ap.add_argument("--dtype", choices=["bf16", "fp16"], default="bf16")
    ap.add_argument("--steps-per-graph", type=int, default=32)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-epoch", action="store_true", help="skip the extra measured full epoch")
    ap.add_argument("--grid", type=int, default=0, help="workgroups per step (0 = per-rank batch, max 256)")
    ap.add_argument("--backend", choices=["auto", "nccl", "gloo"], default="auto",
                    help="process group: auto = RCCL ('nccl') on GPUs; gloo lets ranks share one GPU "
                         "(rehearsal of the multi-rank path; the gradient exchange still runs on the GPU)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist
    from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer
    from csed_514_project_distributed_training_using_pytorch_amd.models import Net
    from csed_514_project_distributed_training_using_pytorch_amd.parallel.comm import (
        all_reduce_max, barrier, init_distributed)
    from csed_514_project_distributed_training_using_pytorch_amd.parallel.sampler import ShardSampler

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    ctx = init_distributed(world_size=world, device="cuda", backend=None if args.backend == "auto" else args.backend)
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float16

    train = synthetic_mnist(60000, seed=0, train=True)
    test = synthetic_mnist(10000, seed=0, train=False)

    def run_once():
        torch.manual_seed(1)
        net = Net().to(ctx.device)
        eng = FusedLeNetTrainer(net, train, lr=0.02, momentum=0.5, global_batch=args.global_batch, ctx=ctx,
                                compute_dtype=dt, grid=args.grid or None)
        sampler = ShardSampler(len(train), ctx.world_size, ctx.rank, shuffle=True, seed=42)
        state = {"epoch": 0, "pos": 0}

        def new_epoch():
            sampler.set_epoch(state["epoch"])
            eng.set_epoch_order(sampler.indices())
            state["epoch"] += 1
            state["pos"] = 0

        def advance(k: int):
            while k > 0:
                if state["pos"] >= eng.full_steps():
                    new_epoch()
                n = min(k, eng.full_steps() - state["pos"])
                eng.run_steps(n, args.steps_per_graph, use_graph=not args.no_graph)
                state["pos"] += n
                k -= n

        new_epoch()
        if not args.no_graph:
            eng.prepare(args.steps_per_graph)
        advance(args.warmup)
        torch.cuda.synchronize(ctx.device)
        eng.take_loss()  # reset the running loss so the reported value covers the timed steps only
        barrier(ctx)
        torch.cuda.synchronize(ctx.device)
        t0 = time.perf_counter()
        advance(args.steps)
        torch.cuda.synchronize(ctx.device)
        barrier(ctx)
        torch.cuda.synchronize(ctx.device)
        elapsed = all_reduce_max(ctx, time.perf_counter() - t0)
        loss_sum, correct = eng.take_loss()

        # one full measured epoch, the reference's quantity: all steps incl. the short last
        # batch + the full 10k validation pass on every rank (ref src/train_dist.py:70-114)
        epoch_s = None
        val = None
        if not args.no_epoch:
            new_epoch()
            torch.cuda.synchronize(ctx.device)
            barrier(ctx)
            te = time.perf_counter()
            eng.run_steps(eng.full_steps(), args.steps_per_graph, use_graph=not args.no_graph)
            eng.last_partial_step()
            vloss, vcorrect = eng.evaluate(test)
            torch.cuda.synchronize(ctx.device)
            barrier(ctx)
            epoch_s = all_reduce_max(ctx, time.perf_counter() - te)
            val = {"val_loss": vloss / len(test), "val_acc": vcorrect / len(test)}
        torch.cuda.synchronize(ctx.device)
        # every rank must agree: one rank's timed-out peer wait invalidates the whole run
        err = int(all_reduce_max(ctx, float(eng.comm_errors())))
        return eng, elapsed, loss_sum, epoch_s, val, err

    eng, elapsed, loss_sum, epoch_s, val, comm_err = run_once()
    comm_retry = None
    if comm_err and os.environ.get("CSED_ALLREDUCE", "auto").lower() != "rccl":
        # a peer wait of the IPC exchange timed out somewhere: free the IPC buffers on every
        # rank and measure again on the process group's all-reduce (RCCL on GPUs), so the
        # reported number is a valid training run rather than a flagged one
        comm_retry = eng.allreduce_kind
        barrier(ctx)
        del eng
        import gc
        gc.collect()
        torch.cuda.synchronize(ctx.device)
        barrier(ctx)
        os.environ["CSED_ALLREDUCE"] = "rccl"
        eng, elapsed, loss_sum, epoch_s, val, comm_err = run_once()
    n = ctx.world_size
    value = args.steps * args.global_batch / elapsed
    base = BASELINE_EPOCH_S.get(n)
    base_ips = 60000.0 / base if base else None
    if ctx.is_main:
        rec = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "images/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 5),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(value / base_ips, 2) if base_ips else None,
            "dtype": args.dtype,
            "data": "synthetic (60000 x 1x28x28 uint8, class-conditional; random-init weights)",
            "config": {"model": "Net (ref src/model.py, 21,840 params)", "global_batch": args.global_batch,
                       "seq_len": None, "parallelism": f"dp{n}", "optimizer": "SGD lr=0.02 momentum=0.5",
                       "engine": "fused HIP (lenet_train + lenet_update"
                                 + {"fused-ipc": " with in-kernel xGMI gradient exchange", "none": ""}.get(
                                     eng.allreduce_kind, " + gradient all-reduce") + ")", "hip_graph": (not args.no_graph) and bool(eng.capture_comm_ok),
                       "allreduce": eng.allreduce_kind, "step": eng.step_kind},
            "epoch_s": round(epoch_s, 4) if epoch_s is not None else None,
            "baseline_epoch_s": base,
            "train_loss_timed_rank0": round(loss_sum / max(1, args.steps * eng.B), 4),
        }
        from csed_514_project_distributed_training_using_pytorch_amd.parallel import ipc as _ipc
        if _ipc.LAST_TIMING:
            rec["config"]["allreduce_select_us"] = _ipc.LAST_TIMING
        if eng.path_timing_us:
            rec["config"]["step_path_select_us"] = eng.path_timing_us
        if comm_retry:
            rec["config"]["comm_retry"] = f"{comm_retry} path timed out; re-measured on the process-group all-reduce"
        if comm_err:
            rec["comm_error"] = "IPC all-reduce timed out waiting for a peer: results invalid"
        if val:
            rec.update({k: round(v, 4) for k, v in val.items()})
        print(json.dumps(rec), flush=True)
    if ctx.is_distributed:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
