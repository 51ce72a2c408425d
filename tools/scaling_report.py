#!/usr/bin/env python3
"""Scaling report: bench.py JSON lines at N = 1/2/4/8 GPUs -> the reference's chart and a table.

The reference's only published result is "time to train 1 epoch vs number of machines"
(ref README.md:20, images/Time to train (1 epoch) vs. Number of machines.png: 17.53 / 11.29 /
7.60 / 5.00 s on 1 / 2 / 4 / 8 CPU VMs, digitised in BASELINE.md).  This turns our bench
records into the same quantity side by side:

    python tools/scaling_report.py BENCH_or_SCALE_files... [--out profiles/scaling] [--title T]

Inputs are any mix of files holding bench JSON lines (one record per line, e.g. logs) or JSON
documents (e.g. the driver's SCALE_rNN.json) in which every dict with "n_gpus" and "value"
keys counts as a record.  For each N the last record wins.  Outputs ``<out>.md`` (table) and
``<out>.png`` (epoch time vs GPUs, log scale, reference overlaid) unless matplotlib is absent.

Columns: images/s (bench ``value``, whole job), ms/step, the warm epoch (``epoch_s``: 938
steps + the 10k validation), the reference's own quantity (``time_elapsed_s``: process start
-> end of epoch-0 validation), the reference time, speed-up on both, and strong-scaling
efficiency value_N / (N * value_1).
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

REF_EPOCH_S = {1: 17.53, 2: 11.29, 4: 7.60, 8: 5.00}  # BASELINE.md (reference README.md:20)


def _walk(obj, out: list) -> None:
    if isinstance(obj, dict):
        if "n_gpus" in obj and "value" in obj:
            out.append(obj)
        for v in obj.values():
            _walk(v, out)
    elif isinstance(obj, list):
        for v in obj:
            _walk(v, out)


def load_records(paths) -> dict[int, dict]:
    recs: list[dict] = []
    for p in paths:
        text = Path(p).read_text()
        try:
            _walk(json.loads(text), recs)
            continue
        except json.JSONDecodeError:
            pass
        for line in text.splitlines():
            line = line.strip()
            if line.startswith("{"):
                try:
                    _walk(json.loads(line), recs)
                except json.JSONDecodeError:
                    continue
    by_n: dict[int, dict] = {}
    for r in recs:
        try:
            by_n[int(r["n_gpus"])] = r
        except (TypeError, ValueError):
            continue
    return dict(sorted(by_n.items()))


def table(by_n: dict[int, dict]) -> list[dict]:
    base = by_n.get(1, {}).get("value")
    rows = []
    for n, r in by_n.items():
        ref = REF_EPOCH_S.get(n)
        ep, te = r.get("epoch_s"), r.get("time_elapsed_s")
        rows.append({
            "n": n, "images_s": r.get("value"), "ms_step": r.get("ms_per_step"), "epoch_s": ep,
            "time_elapsed_s": te, "ref_s": ref,
            "speedup_epoch": ref / ep if ref and ep else None,
            "speedup_time_elapsed": ref / te if ref and te else None,
            "efficiency": r["value"] / (n * base) if base and r.get("value") else None,
            "dtype": r.get("dtype"), "allreduce": (r.get("config") or {}).get("allreduce"),
        })
    return rows


def _f(v, fmt):
    return "-" if v is None else format(v, fmt)


def markdown(rows: list[dict], title: str) -> str:
    out = [f"## {title}", "",
           "| GPUs | images/s | ms/step | epoch s (warm) | time_elapsed s (ref quantity) | reference s | "
           "speed-up (epoch) | speed-up (time_elapsed) | scaling eff. | all-reduce |",
           "|---:|---:|---:|---:|---:|---:|---:|---:|---:|---|"]
    for r in rows:
        out.append(f"| {r['n']} | {_f(r['images_s'], ',.0f')} | {_f(r['ms_step'], '.4f')} | "
                   f"{_f(r['epoch_s'], '.4f')} | {_f(r['time_elapsed_s'], '.3f')} | {_f(r['ref_s'], '.2f')} | "
                   f"{_f(r['speedup_epoch'], ',.0f')}x | {_f(r['speedup_time_elapsed'], '.1f')}x | "
                   f"{_f(r['efficiency'], '.1%')} | {r['allreduce'] or '-'} |")
    out += ["", "Reference: 1 / 2 / 4 / 8 GCP e2-standard-8 CPU VMs, gloo over TCP (BASELINE.md).  Scaling is "
            "strong (global batch 64 split over the GPUs, ref src/train_dist.py:133), so per-GPU work shrinks "
            "to 8 images per step at N = 8."]
    return "\n".join(out) + "\n"


def plot(rows: list[dict], path: Path, title: str) -> bool:
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:
        return False
    fig, ax = plt.subplots(figsize=(6.4, 4.2))
    ns = sorted(REF_EPOCH_S)
    ax.plot(ns, [REF_EPOCH_S[n] for n in ns], "o-", color="gray", label="reference (CPU VMs, gloo)")
    pts = [(r["n"], r["time_elapsed_s"]) for r in rows if r["time_elapsed_s"]]
    if pts:
        ax.plot(*zip(*pts), "s-", color="tab:orange", label="MI355X, process start -> epoch 0 done")
    pts = [(r["n"], r["epoch_s"]) for r in rows if r["epoch_s"]]
    if pts:
        ax.plot(*zip(*pts), "^-", color="tab:blue", label="MI355X, warm epoch (938 steps + validation)")
    ax.set_xscale("log", base=2)
    ax.set_yscale("log")
    ax.set_xticks(ns)
    ax.set_xticklabels([str(n) for n in ns])
    ax.set_xlabel("number of GPUs / machines")
    ax.set_ylabel("time to train 1 epoch (s)")
    ax.set_title(title)
    ax.grid(True, which="both", alpha=0.3)
    ax.legend(fontsize=8)
    path.parent.mkdir(parents=True, exist_ok=True)
    fig.tight_layout()
    fig.savefig(path, dpi=120)
    plt.close(fig)
    return True


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("inputs", nargs="+")
    ap.add_argument("--out", default="profiles/scaling")
    ap.add_argument("--title", default="Time to train 1 epoch vs number of GPUs (MNIST Net, global batch 64)")
    a = ap.parse_args(argv)
    by_n = load_records(a.inputs)
    if not by_n:
        print("no bench records found", file=sys.stderr)
        return 1
    rows = table(by_n)
    out = Path(a.out)
    out.parent.mkdir(parents=True, exist_ok=True)
    md = markdown(rows, a.title)
    out.with_suffix(".md").write_text(md)
    png = plot(rows, out.with_suffix(".png"), a.title)
    print(md)
    if png:
        print(f"wrote {out.with_suffix('.png')}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
