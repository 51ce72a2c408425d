#!/usr/bin/env python3
"""RCCL process-group bring-up on one GPU: the TCPStore rendezvous, init_process_group("nccl",
device_id=...) (torch creates the communicator eagerly when a device is given) and the first
collectives, timed after the HIP context is up.  One rank is the only RCCL configuration a
one-GPU box can run (RCCL refuses two ranks on one GPU); it is the fixed part of an N-rank
communicator's creation, the prediction's ``rccl_init`` term (tools/scaling_report.py).

    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 tools/rccl_init_probe.py
"""
import datetime
import json
import os
import time


def main() -> int:
    import torch
    import torch.distributed as dist

    out = {}
    t = time.perf_counter()
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    torch.empty(1, device=dev).copy_(torch.zeros(1))
    torch.cuda.synchronize(dev)
    out["hip_context_s"] = round(time.perf_counter() - t, 4)
    t = time.perf_counter()
    store, rank, world = next(dist.rendezvous("env://", int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]),
                                              timeout=datetime.timedelta(seconds=120)))
    out["rendezvous_s"] = round(time.perf_counter() - t, 4)
    lazy = "--lazy" in os.sys.argv
    t = time.perf_counter()
    if lazy:  # no device: the communicator is created at the first collective
        dist.init_process_group("nccl", store=store, rank=rank, world_size=world)
    else:
        dist.init_process_group("nccl", store=store, rank=rank, world_size=world, device_id=dev)
    out["init_process_group_s"] = round(time.perf_counter() - t, 4)
    out["lazy"] = lazy
    if lazy:
        t = time.perf_counter()
        g = dist.new_group(backend="gloo")
        out["gloo_subgroup_s"] = round(time.perf_counter() - t, 4)
        y = torch.ones(4)
        t = time.perf_counter()
        dist.all_reduce(y, group=g)
        out["gloo_first_all_reduce_s"] = round(time.perf_counter() - t, 4)
    x = torch.ones(21840, device=dev)
    for name in ("first_broadcast_s", "first_all_reduce_s", "second_all_reduce_s"):
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        if name == "first_broadcast_s":
            dist.broadcast(x, src=0)
        else:
            dist.all_reduce(x)
        torch.cuda.synchronize(dev)
        out[name] = round(time.perf_counter() - t, 4)
    out["world"] = world
    print("RCCL_INIT " + json.dumps(out), flush=True)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
