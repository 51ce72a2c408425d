#!/usr/bin/env python3
"""In-kernel phase stamps of the conv forward kernel (conv_fwd_body's CONV_STAMP: entry, staging
loads issued, LDS stores done, after the barrier, end) at the modular step's shapes: median cycles
per phase over the blocks, and the blocks' start / end spread.

    python tools/conv_stamps.py [--batch 64]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    import torch

    from csed_514_project_distributed_training_using_pytorch_amd.ops import _native

    o = _native.ops()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    B = a.batch
    x0 = torch.randn(B, 1, 28, 28, device=dev, generator=g)
    w1, b1 = torch.randn(10, 1, 5, 5, device=dev, generator=g), torch.randn(10, device=dev, generator=g)
    y1 = torch.empty(B, 10, 12, 12, device=dev, dtype=torch.bfloat16)
    i1 = torch.empty(y1.shape, device=dev, dtype=torch.uint8)
    w2, b2 = torch.randn(20, 10, 5, 5, device=dev, generator=g), torch.randn(20, device=dev, generator=g)
    y2 = torch.empty(B, 20, 4, 4, device=dev, dtype=torch.bfloat16)
    i2 = torch.empty(y2.shape, device=dev, dtype=torch.uint8)
    sc2 = torch.empty(B * 20, device=dev)
    off = torch.zeros(1, device=dev, dtype=torch.long)
    dbg = torch.zeros(B * 32 * 8, device=dev, dtype=torch.long)
    names = ["loads issued", "LDS stores", "barrier", "MFMA + epilogue"]
    for label, fn, nblk in (
            ("conv1 fwd", lambda d: o.conv2d_fwd(x0, w1, b1, y1, 0, i1, None, 2, 1, dbg=d), None),
            ("conv2 fwd", lambda d: o.conv2d_fwd(y1, w2, b2, y2, 0, i2, None, 2, 1, 0.5, 7, 0, off, sc2, d), None)):
        for _ in range(5):
            dbg.zero_()
            fn(dbg)
        torch.cuda.synchronize()
        t = dbg.view(-1, 8).cpu()
        t = t[t[:, 0] > 0]
        d = (t[:, 1:5] - t[:, 0:4]).double()
        med = d.median(0).values.tolist()
        start = (t[:, 0] - t[:, 0].min()).double()
        end = (t[:, 4] - t[:, 0].min()).double()
        print(f"{label}: {len(t)} blocks; median cycles per phase: " +
              ", ".join(f"{n} {m:.0f}" for n, m in zip(names, med)) +
              f"; block start spread p50/max {start.median():.0f}/{start.max():.0f}, end p50/max {end.median():.0f}/{end.max():.0f}",
              flush=True)
    # the weight-gradient blocks of the two backward launches (first image of each block)
    from csed_514_project_distributed_training_using_pytorch_amd.ops.functional import wgrad_workspace_elems
    dy2 = torch.randn(y2.shape, device=dev, generator=g).to(torch.bfloat16)
    dw2, db2, dx2 = torch.empty_like(w2), torch.empty_like(b2), torch.empty_like(y1)
    ws2 = torch.empty(wgrad_workspace_elems(B, 10, 5, 5, 20), device=dev)
    dw1, db1 = torch.empty_like(w1), torch.empty_like(b1)
    ws1 = torch.empty(wgrad_workspace_elems(B, 1, 5, 5, 10), device=dev)
    wnames = ["loads issued", "stores + barrier", "MFMA", "slab write"]
    for label, fn in (
            ("conv2 bwd (wgrad blocks)", lambda d: o.conv2d_bwd(y1, dy2, w2, dw2, db2, ws2, dx2, 0, i2, y2, sc2, 1, d)),
            ("conv1 bwd (wgrad blocks)", lambda d: o.conv2d_bwd(x0, dx2, w1, dw1, db1, ws1, None, 0, i1, y1, None, 1, d))):
        for _ in range(5):
            dbg.zero_()
            fn(dbg)
        torch.cuda.synchronize()
        t = dbg.view(-1, 8).cpu()
        t = t[t[:, 0] > 0]
        d = (t[:, 1:5] - t[:, 0:4]).double()
        med = d.median(0).values.tolist()
        print(f"{label}: {len(t)} blocks; median cycles per phase: " +
              ", ".join(f"{n} {m:.0f}" for n, m in zip(wnames, med)), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
