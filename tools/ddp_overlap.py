"""Time the modular engine's bucketed reducer (parallel/ddp.py) on one GPU: does the per-bucket
all-reduce on the comm stream overlap the rest of backward?  (ref src/train_dist.py:83: torch DDP
fires its all-reduce from backward hooks)

    python tools/ddp_overlap.py [--batch 64] [--steps 200]          # step times per mode
    python tools/ddp_overlap.py --parse <run_kernel_trace.csv>       # overlap from a kernel trace
    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/ddp_overlap.py --trace \
        --mode overlap --bucket-mb 0.01                             # then --parse its csv

One process with an RCCL process group of world 1.  The reducer is forced into its collective path
(``world_size`` set to 2 after construction), so every bucket's all-reduce is issued on the comm
stream from the post-accumulate hooks exactly as at N > 1; the collective is a 1-rank RCCL
all-reduce (no wire time), i.e. this measures the overlap machinery, not xGMI.  Modes:

* ``nocomm``: the reducer's hooks skip communication (``no_sync``);
* ``overlap`` / ``serial``: per-bucket launch from the hooks vs every bucket after backward;
* bucket caps 25 MB (the default: the 87 KB model is one bucket) and 0.01 MB (one bucket per
  parameter tensor of fc1 / conv2 size, several for the smaller ones).
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _modes():
    return [("single", 25.0, True), ("nocomm", 25.0, True), ("overlap", 25.0, True), ("serial", 25.0, False),
            ("overlap", 0.01, True), ("serial", 0.01, False)]


def run(batch: int, steps: int, warmup: int, trace: bool, only=None, graphs=(False, True),
        loader: bool = False) -> list[dict]:
    """Step times of the modular engine (engine/modular.py ModularTrainer: its DDP reducer, fused
    SGD, and -- graph=True -- one HIP-graph replay per step) per reducer mode.  ``loader``: each
    step also gathers a new shuffled batch (data/loader.py DeviceLoader bound to the trainer, i.e.
    the CLI's loop) instead of replaying one fixed batch."""
    import contextlib
    import types

    import torch
    import torch.distributed as dist

    from csed_514_project_distributed_training_using_pytorch_amd import ops
    from csed_514_project_distributed_training_using_pytorch_amd.engine.modular import ModularTrainer
    from csed_514_project_distributed_training_using_pytorch_amd.models.net import Net

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(batch, 1, 28, 28, device=dev, generator=g).to(ops.compute_dtype())
    t = torch.randint(0, 10, (batch,), device=dev, generator=g)
    ctx = types.SimpleNamespace(is_distributed=True, backend="nccl")  # (the reducer's collective path)
    rows = []
    for graph in graphs:
        for mode, cap, overlap in _modes():
            if only is not None and (mode, cap) != only:
                continue
            torch.manual_seed(1)
            net = Net().to(dev).train()
            # single: the one-GPU trainer (no reducer, no grad hooks: src/train.py --engine modular)
            tr = ModularTrainer(net, lr=0.01, momentum=0.5, ctx=None if mode == "single" else ctx, bucket_cap_mb=cap,
                                graph=graph, overlap=overlap)
            if tr.ddp is not None:
                tr.ddp.world_size = 2  # force the collective path (see the module docstring)

            batches = None
            if loader:
                from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist
                from csed_514_project_distributed_training_using_pytorch_amd.data.loader import DeviceLoader

                dl = DeviceLoader(synthetic_mnist(max(64 * batch, 8192), seed=0), batch, shuffle=True, device=dev,
                                  dtype=ops.compute_dtype(), drop_last=True)
                tr.bind_loader(dl)

                def batches_forever():
                    while True:
                        yield from dl

                batches = batches_forever()

            def step():
                xb, tb = next(batches) if batches is not None else (x, t)
                with tr.ddp.no_sync() if mode == "nocomm" and tr.ddp is not None else contextlib.nullcontext():
                    tr.train_batch(xb, tb, clone_loss=False)

            for _ in range(warmup):
                step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if trace:  # phase marker for --phases: the steps window starts after it
                marker = torch.zeros(1, dtype=torch.long, device=dev)
                torch.ops.csed.lenet_add_(marker, 0)
            t0 = time.perf_counter()
            e0.record()
            for _ in range(steps):
                step()
            e1.record()
            if trace:  # ... and ends before this one
                torch.ops.csed.lenet_add_(marker, 0)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / steps
            rows.append({"mode": mode, "graph": graph and tr.use_graph, "batch": batch, "loader": loader, "bucket_mb": cap,
                         "buckets": len(tr.ddp.buckets) if tr.ddp is not None else 0,
                         "us_per_step_gpu": round(e0.elapsed_time(e1) * 1000 / steps, 2),
                         "us_per_step_wall": round(wall * 1e6, 2)})
            for h in (tr.ddp._hooks if tr.ddp is not None else []):
                h.remove()
            del tr
    dist.destroy_process_group()
    return rows


def parse(path: str) -> dict:
    """Comm (RCCL) kernel time and the part of it that overlaps a compute kernel on another stream."""
    ks = []
    with open(path) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]))
    ks.sort()
    comm = [k for k in ks if any(x in k[3].lower() for x in ("nccl", "rccl", "onerankreduce", "allreduce"))]
    comp = [k for k in ks if k not in comm and "rocclr" not in k[3]]
    tot = ov = 0
    for s, e, st, _ in comm:
        tot += e - s
        # union of the other streams' compute intervals intersected with [s, e)
        segs = sorted((max(s, cs), min(e, ce)) for cs, ce, cst, _ in comp if cst != st and cs < e and ce > s)
        cur_s = cur_e = None
        for a, b in segs:
            if cur_e is None or a > cur_e:
                if cur_e is not None:
                    ov += cur_e - cur_s
                cur_s, cur_e = a, b
            else:
                cur_e = max(cur_e, b)
        if cur_e is not None:
            ov += cur_e - cur_s
    names = sorted({k[3] for k in comm})
    return {"comm_kernels": len(comm), "comm_ns": tot, "overlapped_ns": ov,
            "overlap_share": round(ov / tot, 3) if tot else None, "comm_kernel_names": names[:4],
            "streams": sorted({k[2] for k in ks})}


MARKER = "lenet_add_i64_kernel"


def phases(path: str, steps: int) -> dict:
    """Per-kernel stats of a --trace run's kernel trace split at the two phase markers (see run):
    set-up (engine construction, graph capture, warm-up steps) / the timed steps / after, so the
    step's own kernels are not mixed with set-up copies and fills."""
    ks = []
    with open(path) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ks.sort()
    marks = [i for i, k in enumerate(ks) if MARKER in k[2]]
    if len(marks) < 2:
        return {"error": f"found {len(marks)} phase markers ({MARKER}), need 2"}
    a, b = marks[-2], marks[-1]
    out = {}
    for name, sel in (("setup", ks[:a]), ("steps", ks[a + 1:b]), ("after", ks[b + 1:])):
        agg: dict = {}
        for s, e, n in sel:
            c = agg.setdefault(n[:110], [0, 0])
            c[0] += 1
            c[1] += e - s
        out[name] = {"kernels": len(sel), "busy_us": round(sum(v[1] for v in agg.values()) / 1e3, 2),
                     "by_kernel": {n: {"calls": v[0], "total_us": round(v[1] / 1e3, 2),
                                       "per_step_calls": round(v[0] / steps, 2) if name == "steps" else None,
                                       "avg_us": round(v[1] / v[0] / 1e3, 3)}
                                   for n, v in sorted(agg.items(), key=lambda kv: -kv[1][1])}}
    st = ks[a + 1:b]
    if st:
        out["steps"]["window_us"] = round((st[-1][1] - st[0][0]) / 1e3, 2)
        out["steps"]["us_per_step"] = round((st[-1][1] - st[0][0]) / 1e3 / steps, 2)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--trace", action="store_true", help="short run of one mode for a kernel trace")
    ap.add_argument("--mode", default="overlap", help="--trace: nocomm / overlap / serial")
    ap.add_argument("--bucket-mb", type=float, default=0.01, help="--trace: bucket cap")
    ap.add_argument("--parse", help="run_kernel_trace.csv of a --trace run")
    ap.add_argument("--phases", help="run_kernel_trace.csv of a --trace run: per-kernel stats of set-up vs steps")
    ap.add_argument("--graph", choices=["both", "eager", "graph"], default="both")
    ap.add_argument("--loader", action="store_true", help="gather a new batch per step (bound DeviceLoader)")
    ap.add_argument("--only", help="MODE:BUCKET_MB, e.g. single:25 -- time that mode only")
    a = ap.parse_args()
    if a.parse:
        print(json.dumps(parse(a.parse)))
        return
    if a.phases:
        print(json.dumps(phases(a.phases, 20), indent=1))
        return
    only = None
    if a.only:
        m, c = a.only.split(":")
        only = (m, float(c))
    if a.trace:
        a.steps, a.warmup, only = 20, 5, (a.mode, a.bucket_mb)
    graphs = {"both": (False, True), "eager": (False,), "graph": (True,)}[a.graph]
    for r in run(a.batch, a.steps, a.warmup, a.trace, only, graphs, a.loader):
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
