#!/usr/bin/env python3
"""Soak of the round-4 one-off divergence (profiles/dp_exchange_r4.md §3: the world-8 looped-back
exact-fp32 run once ended 0.14 away from world 1 with a clean timeout word).

Runs the three-way comparison of tests/test_exchange_loopback_gpu.py many times in ONE process:
per round two world-1 runs (must be bitwise equal: otherwise the training kernel is
nondeterministic) and one world-8 looped-back run with the in-kernel invariant on (every received
word must bit-equal the pushed one; a violation names the word).  One JSON line per round, then a
summary.  A failing round is recorded, not retried.

    python tools/loopback_soak.py [--rounds 20] [--steps 16]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["CSED_LOOPBACK_CHECK"] = "1"

import torch  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402


def run(world: int, data, steps: int, seed: int):
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    eng = FusedLeNetTrainer(Net().to(dev), data, lr=0.05, momentum=0.5, global_batch=8, compute_dtype=torch.float32,
                            loopback_world=world)
    eng.set_epoch_order(torch.randperm(len(data), generator=torch.Generator().manual_seed(seed)))
    eng.run_steps(steps, steps_per_graph=8)
    torch.cuda.synchronize()
    err, diag = eng.comm_errors(), eng.comm_diag()
    out = eng.flat.data.clone()
    eng.close()
    return out, err, diag


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--steps", type=int, default=16)
    a = ap.parse_args()
    data = synthetic_mnist(2048, seed=3)
    bad = 0
    worst = 0.0
    for r in range(a.rounds):
        seed = 1 + (r % 4)
        l1, e1, _ = run(0, data, a.steps, seed)
        w8, e8, d8 = run(8, data, a.steps, seed)
        l2, e2, _ = run(0, data, a.steps, seed)
        rel = float((w8 - l1).norm() / l1.norm())
        det = bool(torch.equal(l1, l2))
        ok = det and e8 == 0 and rel < 1e-3
        bad += not ok
        worst = max(worst, rel)
        print(json.dumps({"round": r, "order_seed": seed, "world1_deterministic": det, "world8_rel": rel,
                          "world8_error_word": e8, "first_mismatch": d8, "ok": ok}), flush=True)
    print(json.dumps({"rounds": a.rounds, "failed": bad, "worst_world8_rel": worst}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
