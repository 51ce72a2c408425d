"""Data-parallel self-check, one rank per GPU: the reference's DDP step (ref
src/train_dist.py:63 DDP wrap, :83 backward -> gradient all-reduce, :146 process group)
run through this framework's production path and checked against its fallback.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        -m csed_514_project_distributed_training_using_pytorch_amd.parallel.dpcheck [--steps K]

On GPUs (RCCL process group, one rank per GPU) every rank:

1. records ``hipDeviceCanAccessPeer`` for every ordered pair of the job's GPUs;
2. trains K exact-fp32 steps on the fused engine in ``auto`` mode (the in-kernel IPC
   exchange over xGMI, kept only if its self-test passes and it times faster than RCCL);
3. trains the same K steps from the same initial state with ``CSED_ALLREDUCE=rccl``
   (reduce-only update -> RCCL all-reduce -> SGD kernel);
4. checks: the exchange's error word is 0, replicas are bitwise identical in both runs
   (parameters and momentum), and the two runs agree -- bitwise at world 2 (a + b is
   order-free), to fp32 summation-order tolerance above that (RCCL's ring does not sum
   in rank order).

Rank 0 prints one ``DPCHECK {json}`` line (with every rank's ``exchange_diag``: peer access, IPC
open, self-test, path timing, error word, first mismatch -- parallel/ipc.py DIAG_KEYS); the exit
code is nonzero if a check failed.
``--device cpu`` runs the same launch / rendezvous / replica-check plumbing on gloo with the
modular (per-op) engine.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

from .comm import init_distributed, replica_checksum
from .ipc import empty_diag, gather_diag


def _gpu_run(ctx, data, steps: int, mode: str, dtype: torch.dtype) -> dict:
    from ..engine.fused import FusedLeNetTrainer
    from ..models import Net
    from .sampler import ShardSampler

    os.environ["CSED_ALLREDUCE"] = mode
    torch.manual_seed(1)
    eng = FusedLeNetTrainer(Net().to(ctx.device), data, lr=0.05, momentum=0.5, global_batch=64, ctx=ctx,
                            compute_dtype=dtype)
    smp = ShardSampler(len(data), ctx.world_size, ctx.rank, shuffle=True, seed=42)
    smp.set_epoch(0)
    eng.set_epoch_order(smp.indices())
    eng.run_steps(steps, steps_per_graph=8)
    torch.cuda.synchronize(ctx.device)
    err = eng.comm_errors()
    same_p, _, _ = replica_checksum(ctx, eng.flat.data)
    same_m, _, _ = replica_checksum(ctx, eng.momentum_buf)
    out = {"allreduce": eng.allreduce_kind, "note": eng.exchange_note, "path_timing_us": eng.path_timing_us,
           "error_word": err, "replicas_identical": bool(same_p and same_m),
           "finite": bool(torch.isfinite(eng.flat.data).all()), "params": eng.flat.data.clone(),
           # every rank's stage results (parallel/ipc.py DIAG_KEYS): names a failing stage / rank
           "exchange_diag": gather_diag(ctx, eng.exchange_diag())}
    eng.close()
    return out


def check(args) -> tuple[bool, dict]:
    ctx = init_distributed(device=args.device, backend=None if args.backend == "auto" else args.backend)
    world = ctx.world_size
    rec: dict = {"world": world, "device": args.device, "backend": ctx.backend, "steps": args.steps}
    ok = True
    if args.device == "cuda":
        from ..data import synthetic_mnist

        n = torch.cuda.device_count()
        devs = sorted({(r % n) for r in range(world)})
        rec["gpus"] = len(devs)
        rec["peer_access"] = {f"{i}->{j}": bool(torch.cuda.can_device_access_peer(i, j))
                              for i in devs for j in devs if i != j}
        data = synthetic_mnist(4096, seed=3)
        dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}[args.dtype]
        fused = _gpu_run(ctx, data, args.steps, "auto", dtype)
        rccl = _gpu_run(ctx, data, args.steps, "rccl", dtype)
        p_f, p_r = fused.pop("params"), rccl.pop("params")
        rel = float((p_f - p_r).norm() / p_r.norm())
        bitwise = bool(torch.equal(p_f, p_r))
        rec.update(fused=fused, rccl=rccl, fused_vs_rccl_rel=rel, fused_equals_rccl_bitwise=bitwise)
        ok &= fused["error_word"] == 0 and fused["replicas_identical"] and fused["finite"]
        ok &= rccl["replicas_identical"] and rccl["finite"] and rccl["allreduce"] == "rccl"
        # (ranks sharing a GPU: the GPU pairs above are empty and "gpus" counts the distinct GPUs)
        if fused["allreduce"] == "fused-ipc" and world == 2:
            ok &= bitwise
        else:
            ok &= rel < args.tol
        if args.require_fused:
            ok &= fused["allreduce"] == "fused-ipc"
    else:
        from ..data import DeviceLoader, synthetic_mnist
        from ..engine.modular import ModularTrainer
        from ..models import Net
        from .sampler import ShardSampler

        data = synthetic_mnist(1024, seed=3)
        torch.manual_seed(1)
        tr = ModularTrainer(Net(), lr=0.05, momentum=0.5, ctx=ctx, loss="ce")
        smp = ShardSampler(len(data), world, ctx.rank, shuffle=True, seed=42)
        it = iter(DeviceLoader(data, 64 // world, sampler=smp, device=ctx.device))
        for _ in range(args.steps):
            tr.train_batch(*next(it))
        flat = torch.cat([p.detach().reshape(-1) for p in tr.model.parameters()])
        same, _, _ = replica_checksum(ctx, flat)
        rec.update(allreduce=f"process group ({ctx.backend})", replicas_identical=bool(same),
                   exchange_diag=gather_diag(ctx, dict(empty_diag(ctx), allreduce=f"process group ({ctx.backend})",
                                                       note="CPU plumbing run: no exchange")))
        ok &= bool(same)
    rec["ok"] = bool(ok)
    # every rank's verdict: the job passes only if all do
    t = torch.tensor([1 if ok else 0], dtype=torch.int32,
                     device=ctx.device if ctx.backend == "nccl" else torch.device("cpu"))
    if ctx.is_distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
    rec["all_ranks_ok"] = bool(t.item())
    return bool(t.item()), rec


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda")
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--backend", choices=["auto", "nccl", "gloo"], default="auto",
                    help="gloo: ranks may share one GPU (the rehearsal of the one-rank-per-GPU check)")
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--tol", type=float, default=1e-4, help="fused vs RCCL relative tolerance (world > 2)")
    ap.add_argument("--require-fused", action="store_true", help="fail unless the fused exchange is kept")
    args = ap.parse_args(argv)
    ok, rec = check(args)
    if int(os.environ.get("RANK", "0")) == 0:
        print("DPCHECK " + json.dumps(rec), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
