#!/usr/bin/env python3
"""Phase stamps of the fused MLP head (ops.mlp_head_nll's one forward launch) at the reference's
batch: median s_memtime cycles per phase over blocks (diagnostics for profiles/round5.md).

    python tools/mlp_stamps.py [--batch 64]
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
    x = torch.randn(B, 320, device=dev, generator=g).relu().to(torch.bfloat16)
    w1, b1 = torch.randn(50, 320, device=dev, generator=g) * 0.05, torch.randn(50, device=dev, generator=g)
    w2, b2 = torch.randn(10, 50, device=dev, generator=g) * 0.2, torch.randn(10, device=dev, generator=g)
    t = torch.randint(0, 10, (B,), device=dev, generator=g)
    h = torch.empty(B, 50, device=dev, dtype=torch.bfloat16)
    logp, out = torch.empty(B, 10, device=dev), torch.empty((), device=dev)
    nb = (B + 15) // 16
    part, cnt = torch.empty(nb, device=dev), torch.zeros(1, device=dev, dtype=torch.int64)
    off = torch.zeros(1, device=dev, dtype=torch.long)
    dbg = torch.zeros(nb * 8, device=dev, dtype=torch.long)
    for _ in range(5):
        o.mlp_head_fwd(x, w1, b1, 2, 0.5, 7, 1, off, h, w2, b2, t, logp, out, part, cnt, 1, 1, dbg)
    torch.cuda.synchronize()
    st = dbg.view(nb, 8).cpu()
    names = ["operand loads + fc1 MFMAs", "partials + barrier", "fc1 epilogue (dropout) + h stores",
             "barrier", "head MFMA + barrier", "head epilogue + loss hand-off"]
    d = [(st[:, i + 1] - st[:, i]).float().median().item() for i in range(6)]
    print(f"batch {B}, {nb} blocks; median cycles: " + ", ".join(f"{n} {v:.0f}" for n, v in zip(names, d)))
    print(f"total (stamp 0 -> 6, wave 0 of each block): {(st[:, 6] - st[:, 0]).float().median().item():.0f}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
