#!/usr/bin/env python3
"""Per-op launch times of the modular (per-op) step's kernels at the reference's batch (B = 64,
bf16 compute): each op is captured REPS times back to back in one HIP graph and replayed, so a
number is one launch's share of a dependent chain -- its kernel time plus the graph's launch gap,
as inside the engine's step graph -- without a tracer's overhead.  Pick the extension build with
CSED_NATIVE_SO (same-box A/B of builds).

    python tools/op_probe.py [--batch 64] [--reps 50] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()

    import torch

    from csed_514_project_distributed_training_using_pytorch_amd.ops import _native
    from csed_514_project_distributed_training_using_pytorch_amd.ops.functional import wgrad_workspace_elems

    o = _native.ops()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    B, bf = a.batch, torch.bfloat16
    r = lambda *s, dt=torch.float32: torch.randn(*s, device=dev, generator=g).to(dt)  # noqa: E731
    x0 = r(B, 1, 28, 28)
    w1, b1 = r(10, 1, 5, 5) * 0.2, r(10)
    y1 = torch.empty(B, 10, 12, 12, device=dev, dtype=bf)
    i1 = torch.empty(y1.shape, device=dev, dtype=torch.uint8)
    w2, b2 = r(20, 10, 5, 5) * 0.1, r(20)
    y2 = torch.empty(B, 20, 4, 4, device=dev, dtype=bf)
    i2 = torch.empty(y2.shape, device=dev, dtype=torch.uint8)
    sc2 = torch.empty(B * 20, device=dev)
    off = torch.zeros(1, device=dev, dtype=torch.long)
    wf1, bf1 = r(50, 320) * 0.05, r(50)
    h = torch.empty(B, 50, device=dev, dtype=bf)
    wf2, bf2 = r(10, 50) * 0.1, r(10)
    t = torch.randint(0, 10, (B,), device=dev, generator=g)
    logp, loss = torch.empty(B, 10, device=dev), torch.empty((), device=dev)
    part, cnt = torch.empty((B + 15) // 16, device=dev), torch.zeros(1, device=dev, dtype=torch.int64)
    gout = torch.ones((), device=dev)
    dh, dwf2, dbf2 = torch.empty_like(h), torch.empty_like(wf2), torch.empty(10, device=dev)
    dp2, dwf1, dbf1 = torch.empty(B, 320, device=dev, dtype=bf), torch.empty_like(wf1), torch.empty(50, device=dev)
    ws2 = torch.empty(wgrad_workspace_elems(B, 10, 5, 5, 20), device=dev)
    ws1 = torch.empty(wgrad_workspace_elems(B, 1, 5, 5, 10), device=dev)
    dw2, db2, dx2 = torch.empty_like(w2), torch.empty_like(b2), torch.empty_like(y1)
    dw1, db1 = torch.empty_like(w1), torch.empty_like(b1)
    flat = r(21840)
    gflat, mom = r(21840), torch.zeros(21840, device=dev)
    step, ticket = torch.zeros(1, device=dev, dtype=torch.long), torch.zeros(1, device=dev, dtype=torch.int32)
    tiny = torch.empty(1, device=dev)

    ops = {
        "trivial (channel_mask n=1)": lambda: o.channel_mask(tiny, 0.5, 1, 0, None),
        "conv1 fwd+pool (fp32 in)": lambda: o.conv2d_fwd(x0, w1, b1, y1, 0, i1, None, 2, 1),
        "conv2 fwd+dropout2d+pool": lambda: o.conv2d_fwd(y1, w2, b2, y2, 0, i2, None, 2, 1, 0.5, 7, 0, off, sc2),
        "fc1 fwd (relu+dropout)": lambda: o.gemm(y2.view(B, 320), wf1.t(), h, bf1, 1.0, 0.0, 2, 0.5, 7, 1, off,
                                                 None, 1.0, 1),
        "head fwd (fc2+lsm+nll)": lambda: o.linear_lsm_nll_fwd(h, wf2, bf2, t, logp, loss, part, cnt, 1, 1),
        "fc1 + head fwd (one launch)": lambda: o.mlp_head_fwd(y2.view(B, 320), wf1, bf1, 2, 0.5, 7, 1, off, h, wf2,
                                                              bf2, t, logp, loss, part, cnt, 1, 1),
        "head bwd (pair)": lambda: o.linear_bwd(logp, h, wf2, None, 1.0, dh, dwf2, dbf2, 1, t, gout, float(B)),
        "fc1 bwd (pair)": lambda: o.linear_bwd(dh, y2.view(B, 320), wf1, h, 2.0, dp2, dwf1, dbf1, 1),
        "head + fc1 bwd (one launch)": lambda: o.mlp_head_bwd(logp, t, gout, float(B), h, y2.view(B, 320), wf1, wf2,
                                                              2.0, dp2, dwf1, dbf1, dwf2, dbf2, 1),
        "conv2 bwd (wgrad+dgrad+reduce)": lambda: o.conv2d_bwd(y1, dp2.view(B, 20, 4, 4), w2, dw2, db2, ws2, dx2, 0,
                                                              i2, y2, sc2, 1),
        "conv1 bwd (wgrad+reduce)": lambda: o.conv2d_bwd(x0, dx2, w1, dw1, db1, ws1, None, 0, i1, y1, None, 1),
        "conv2 bwd, reduce deferred": lambda: o.conv2d_bwd(y1, dp2.view(B, 20, 4, 4), w2, dw2, db2, ws2, dx2, 0,
                                                          i2, y2, sc2, 1, defer_reduce=True),
        "conv1 bwd carrying conv2's reduce": lambda: o.conv2d_bwd(x0, dx2, w1, dw1, db1, ws1, None, 0, i1, y1, None, 1,
                                                                 carry_ws=ws2, carry_dw=dw2, carry_db=db2, carry_n=B,
                                                                 carry_ic=10, carry_kh=5, carry_kw=5),
        "sgd (21840)": lambda: o.sgd_flat(flat, gflat, mom, 0.01, 0.5, 0.0, 0.0, False, 1.0, step, ticket),
    }
    s = torch.cuda.Stream()
    res = {}
    for name, fn in ops.items():
        with torch.cuda.stream(s):
            for _ in range(3):
                fn()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            for _ in range(a.reps):
                fn()
        graph.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            graph.replay()
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) * 1000 / (a.iters * a.reps), 2)
        print(f"{name:34s} {res[name]:7.2f} us/launch", flush=True)
    print(json.dumps({"batch": B, "us_per_launch": res, "so": os.environ.get("CSED_NATIVE_SO", "in-tree")}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
