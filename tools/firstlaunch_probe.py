#!/usr/bin/env python3
"""First-call vs second-call host cost of every GPU operation the bench's reference span runs
(fresh process): the HIP runtime loads a kernel's code object (one per compiled translation unit
-- torch's and ours) lazily, at that TU's first launch, so a cold epoch pays every load it has
not paid before.  Prints one JSON line: {op: [first_ms, second_ms]}, in order.

    python tools/firstlaunch_probe.py [--preload]

--preload calls csed::preload_kernels (csrc/bindings.cpp) first and reports its own time."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    t0 = time.perf_counter()
    import torch

    from csed_514_project_distributed_training_using_pytorch_amd.data.mnist import synthetic_mnist
    from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer
    from csed_514_project_distributed_training_using_pytorch_amd.models import Net
    from csed_514_project_distributed_training_using_pytorch_amd.ops import _native

    out = {"import_s": round(time.perf_counter() - t0, 3)}
    dev = torch.device("cuda", 0)

    def timed(name, fn, reps=2):
        res = []
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize(dev)
            res.append(round(1e3 * (time.perf_counter() - t), 3))
        out[name] = res

    t = time.perf_counter()
    torch.cuda.set_device(dev)
    out["set_device_ms"] = round(1e3 * (time.perf_counter() - t), 3)
    timed("first_h2d_copy", lambda: torch.empty(1, device=dev).copy_(torch.zeros(1)))
    _native.require()
    if "--preload" in sys.argv:
        timed("preload_kernels", lambda: torch.ops.csed.preload_kernels(0))
    timed("torch_zeros", lambda: torch.zeros(1000, device=dev))
    a = torch.randn(1000, device=dev)
    timed("torch_clone", lambda: a.clone())
    timed("torch_copy_", lambda: a.copy_(a.clone()))
    timed("torch_sum_double", lambda: a.view(500, 2).double().sum(0).tolist())
    timed("d2h_cpu", lambda: a.cpu())
    torch.manual_seed(1)
    train = synthetic_mnist(4096, seed=0)
    test = synthetic_mnist(10000, seed=0, train=False)
    net = Net().to(dev)
    t = time.perf_counter()
    eng = FusedLeNetTrainer(net, train, lr=0.02, momentum=0.5, global_batch=64)
    torch.cuda.synchronize(dev)
    out["engine_ms"] = round(1e3 * (time.perf_counter() - t), 3)
    out["engine_bringup_s"] = {k: round(v, 4) for k, v in eng.bringup_s.items()}
    eng.set_epoch_order(torch.randperm(4096))
    timed("step", eng.step)
    timed("evaluate_10k", lambda: eng.evaluate(test))
    t = time.perf_counter()
    eng.prepare(32, ks=(63,))
    torch.cuda.synchronize(dev)
    out["prepare_ms"] = round(1e3 * (time.perf_counter() - t), 3)
    out["capture_stamps_s"] = {k: round(v, 4) for k, v in eng.bringup_s.items() if k.startswith("capture")}
    g = eng.graph(32)
    timed("replay32", g.replay, reps=3)
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
