#!/usr/bin/env python3
"""Wall time of K graph-replayed training steps launched as different graph splits, the way
bench.py's timed window measures them (device idle -> host launches -> synchronize): one K-step
graph vs a small first graph followed by the rest.  A HIP graph's launch submits its kernel nodes
one by one from the host; while that runs the device can already execute a short first graph.

    python tools/launch_ramp_probe.py [--batch 64] [--steps 20] [--reps 30]

Prints one JSON line: {split: median_us_per_step}."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    import torch

    from csed_514_project_distributed_training_using_pytorch_amd.data.mnist import synthetic_mnist
    from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer
    from csed_514_project_distributed_training_using_pytorch_amd.models import Net

    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    eng = FusedLeNetTrainer(Net().to(dev), synthetic_mnist(60000, seed=0), lr=0.02, momentum=0.5,
                            global_batch=a.batch)
    eng.set_epoch_order(torch.randperm(60000))
    K = a.steps
    splits = {"one": [K]}
    for first in (1, 2, 4):
        splits[f"{first}+{K - first}"] = [first, K - first]
    if K > 10:
        splits[f"2+8+{K - 10}"] = [2, 8, K - 10]
    graphs = {n: eng.graph(n) for sp in splits.values() for n in sp}
    out = {}
    order = torch.randperm(60000)
    for rep in range(a.reps):
        eng.set_epoch_order(order)  # (every rep from the epoch start: the cursor stays in range)
        for name, sp in splits.items():
            plan = [graphs[n].replay for n in sp]
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for launch in plan:
                launch()
            torch.cuda.synchronize(dev)
            out.setdefault(name, []).append((time.perf_counter() - t0) * 1e6 / K)
    res = {k: round(sorted(v)[len(v) // 2], 3) for k, v in out.items()}
    res["batch"], res["steps"] = a.batch, K
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
