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

Prediction (``--predict``, on by default).  At global batch 64 each of N ranks runs a step of
per-rank batch 64/N whose exchange pushes to N-1 peers.  Both parts were measured on one GPU
with the exchange looped back to N virtual ranks (``tools/exchange_loopback.py``,
profiles/dp_exchange_r4.md): ``LOOPBACK_STEP_US[(B, N)]`` is that graph-replayed
step.  The loopback push never leaves the device, so the predicted N-GPU step adds one xGMI
one-way hop (``--hop-us``, 1 us assumed) and the time the pushes occupy one link: every rank
sends each peer its whole live gradient as LL words (21,840 x 8 bytes = 175 KB, one link per
peer, all links at once), ``wire = 175 KB / --link-gbs`` (153 GB/s per link assumed: 1.14 us;
no overlap with the update's compute is credited, so this term is an upper bound).  The
predicted epoch keeps the N=1 record's non-step remainder (validation + tail):

    step_N  = LOOPBACK_STEP_US[(64 / N, N)] + hop + wire   (N > 1; N = 1: no exchange)
    epoch_N = 938 * step_N + (epoch_s_1 - 938 * ms_per_step_1)

A loopback log (``--loopback-log``, the ``B=.. N=.. ... step X us`` lines of
exchange_loopback.py) replaces the built-in table.  The driver's SCALE record is then checked
against the prediction in the ``measured / predicted`` column.

Predicted ``time_elapsed`` (the reference's own quantity: its t0, taken right after its imports,
-> end of epoch-0 validation, ref src/train_dist.py:1-11,119,112; bench.py takes t0 after
``import torch`` and the package, so the imports are outside it and inside
``process_elapsed_s``).  bench.py's ``bringup_s`` splits it into phases (max over ranks).  For
N ranks:

    time_elapsed_N = process_group_N                           (--cpu-bringup: bench.py --gpus N
                                                                 --device cpu on the GPU box: an
                                                                 N-rank rendezvous)
                   + data_wait_1 + engine_1 + capture_1 + test_upload_1     (the N = 1 GPU record)
                   + exchange bring-up (engine.ipc_open + engine.self_test + engine.path_timing of
                     --rehearsal, a 2-rank gloo run sharing the GPU; 0 at N = 1)
                   + epoch0_1 + 938 * (step_N - step_1)        (the epoch at the predicted step)

Records from before round 5 (an ``import`` phase, no ``import_torch``) measured time_elapsed_s
from process start; for those the prediction keeps spawn + import in the span.

What it leaves out: RCCL's communicator set-up over N GPUs (the CPU rehearsal's rendezvous is
gloo) and xGMI peer mapping (the rehearsal maps one GPU's memory).
"""
from __future__ import annotations

import argparse
import json
import re
import sys
from pathlib import Path

REF_EPOCH_S = {1: 17.53, 2: 11.29, 4: 7.60, 8: 5.00}  # BASELINE.md (reference README.md:20)
STEPS_PER_EPOCH = 938
GLOBAL_BATCH = 64
# graph-replayed lenet_train + lenet_update step (us) at per-rank batch B with the in-kernel
# exchange looped back to N virtual ranks, one MI355X (profiles/r4/exchange_loopback_r4f7.log,
# profiles/dp_exchange_r4.md)
LOOPBACK_STEP_US = {  # round 6 (profiles/r6/rehearsal/r6i_loopback.log)
    (8, 1): 12.34, (8, 2): 13.51, (8, 4): 13.97, (8, 8): 14.59,
    (16, 1): 12.37, (16, 2): 13.66, (16, 4): 13.96, (16, 8): 14.71,
    (32, 1): 12.71, (32, 2): 13.88, (32, 4): 14.19, (32, 8): 14.92,
    (64, 1): 13.43, (64, 2): 14.53, (64, 4): 14.94, (64, 8): 15.71,
}
WIRE_BYTES = 21840 * 8  # live exchange words per peer per step (lenet_fused.hip ll_push)
_LB_LINE = re.compile(r"B=\s*(\d+)\s+N=(\d+).*?step\s+([0-9.]+)\s*us")


def load_loopback(path) -> dict[tuple[int, int], float]:
    """(per-rank B, N) -> step us from exchange_loopback.py output."""
    out = {}
    for line in Path(path).read_text().splitlines():
        m = _LB_LINE.search(line)
        if m:
            out[(int(m.group(1)), int(m.group(2)))] = float(m.group(3))
    return out


def predict(by_n: dict[int, dict], steps_us: dict, hop_us: float, ns=(1, 2, 4, 8),
            wire_us: float = 0.0) -> dict[int, dict]:
    """Predicted per-N step (us), images/s and warm epoch (s) at global batch 64."""
    r1 = by_n.get(1) or {}
    rest = None
    if r1.get("epoch_s") and r1.get("ms_per_step"):
        rest = max(0.0, r1["epoch_s"] - STEPS_PER_EPOCH * r1["ms_per_step"] * 1e-3)
    out = {}
    for n in ns:
        b = GLOBAL_BATCH // n
        if (b, n) not in steps_us:
            continue
        step = steps_us[(b, n)] + (hop_us + wire_us if n > 1 else 0.0)
        out[n] = {"step_us": step, "images_s": GLOBAL_BATCH / (step * 1e-6),
                  "epoch_s": STEPS_PER_EPOCH * step * 1e-6 + rest if rest is not None else None}
    return out


def load_rccl_init(path) -> dict | None:
    """The ``RCCL_INIT {json}`` line of tools/rccl_init_probe.py."""
    for line in Path(path).read_text().splitlines():
        if line.startswith("RCCL_INIT "):
            return json.loads(line[len("RCCL_INIT "):])
    return None


def predict_time_elapsed(by_n: dict[int, dict], pred: dict[int, dict], cpu_by_n: dict[int, dict],
                         rehearsal: dict | None, rccl: dict | None = None,
                         terms: dict | None = None) -> dict[int, float]:
    """Predicted time_elapsed_s per N (the module docstring's formula); every term comes from a
    record, and ``terms`` (if given) receives them per N for the report."""
    r1 = by_n.get(1) or {}
    ph1 = r1.get("bringup_s") or {}
    if not ph1 or not r1.get("epoch0_s") or 1 not in pred:
        return {}
    base = sum(ph1.get(k, 0.0) for k in ("data_wait", "engine", "capture", "test_upload"))
    ctx1 = ph1.get("process_group", 0.0)  # N = 1: the wait for this rank's HIP-context thread
    xb = 0.0
    if rehearsal:
        rph = rehearsal.get("bringup_s") or {}
        xb = sum(rph.get(k, 0.0) for k in ("engine.ipc_open", "engine.self_test", "engine.path_timing"))
    rinit = (rccl.get("init_process_group_s", 0.0) + rccl.get("first_broadcast_s", 0.0)) if rccl else 0.0
    out = {}
    for n, p in pred.items():
        if n == 1:
            launch, rdzv = ctx1, 0.0
        else:
            c = (cpu_by_n.get(n) or {}).get("bringup_s")
            if not c:
                continue
            # the rendezvous (N concurrent processes, their import skew) overlaps the HIP context's
            # creation (bench.py: store barrier in the main thread, context in its own), then the
            # RCCL communicator is created on the store
            rdzv = c.get("rendezvous", c.get("process_group", 0.0))
            # then the process group on that store: lazy RCCL + the gloo control group (what the CPU
            # record's process_group adds to its rendezvous: a gloo group over N ranks); an eager
            # RCCL communicator (bench.py --eager-rccl) adds --rccl-init on top
            pg_init = max(0.0, c.get("process_group", 0.0) - c.get("rendezvous", 0.0)) if "rendezvous" in c else 0.0
            # (rendezvous and the lazy process group both run in the main thread, beside the HIP-
            # context thread: bench.py bring-up)
            launch = max(ctx1, rdzv + pg_init) + rinit
        ep0 = r1["epoch0_s"] + STEPS_PER_EPOCH * (p["step_us"] - pred[1]["step_us"]) * 1e-6
        out[n] = launch + base + (xb if n > 1 else 0.0) + ep0
        if terms is not None:
            terms[n] = {"hip_ctx_wait_1": ctx1, "rendezvous_N": rdzv,
                        "pg_init_N": (max(0.0, (cpu_by_n.get(n) or {}).get("bringup_s", {}).get("process_group", 0.0)
                                          - (cpu_by_n.get(n) or {}).get("bringup_s", {}).get("rendezvous", 0.0))
                                      if n > 1 else 0.0),
                        "rccl_init": rinit if n > 1 else 0.0,
                        "setup_1 (data_wait+engine+capture+test_upload)": base,
                        "exchange_bringup (ipc_open+self_test+path_timing)": xb if n > 1 else 0.0,
                        "epoch0_N": ep0, "total": out[n]}
    return out


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


def table(by_n: dict[int, dict], pred: dict[int, dict] | None = None) -> list[dict]:
    base = by_n.get(1, {}).get("value")
    pred = pred or {}
    rows = []
    for n in sorted(set(by_n) | set(pred)):
        r = by_n.get(n, {"value": None})
        p = pred.get(n, {})
        ref = REF_EPOCH_S.get(n)
        ep, te = r.get("epoch_s"), r.get("time_elapsed_s")
        rows.append({
            "n": n, "images_s": r.get("value"), "ms_step": r.get("ms_per_step"), "epoch_s": ep,
            "time_elapsed_s": te, "ref_s": ref,
            "speedup_epoch": ref / ep if ref and ep else None,
            "speedup_time_elapsed": ref / te if ref and te else None,
            "efficiency": r["value"] / (n * base) if base and r.get("value") else None,
            "dtype": r.get("dtype"), "allreduce": (r.get("config") or {}).get("allreduce"),
            "pred_images_s": p.get("images_s"), "pred_epoch_s": p.get("epoch_s"),
            "pred_time_elapsed_s": p.get("time_elapsed_s"),
            "vs_pred": r["value"] / p["images_s"] if r.get("value") and p.get("images_s") else None,
        })
    return rows


def _f(v, fmt):
    return "-" if v is None else format(v, fmt)


def markdown(rows: list[dict], title: str) -> str:
    out = [f"## {title}", "",
           "| GPUs | images/s | ms/step | epoch s (warm) | time_elapsed s (ref quantity) | reference s | "
           "speed-up (epoch) | speed-up (time_elapsed) | scaling eff. | all-reduce | predicted images/s | "
           "predicted epoch s | predicted time_elapsed s | measured / predicted |",
           "|---:|---:|---:|---:|---:|---:|---:|---:|---:|---|---:|---:|---:|---:|"]
    for r in rows:
        out.append(f"| {r['n']} | {_f(r['images_s'], ',.0f')} | {_f(r['ms_step'], '.4f')} | "
                   f"{_f(r['epoch_s'], '.4f')} | {_f(r['time_elapsed_s'], '.3f')} | {_f(r['ref_s'], '.2f')} | "
                   f"{_f(r['speedup_epoch'], ',.0f')}x | {_f(r['speedup_time_elapsed'], '.1f')}x | "
                   f"{_f(r['efficiency'], '.1%')} | {r['allreduce'] or '-'} | {_f(r['pred_images_s'], ',.0f')} | "
                   f"{_f(r['pred_epoch_s'], '.4f')} | {_f(r.get('pred_time_elapsed_s'), '.3f')} | "
                   f"{_f(r['vs_pred'], '.2f')} |")
    out += ["", "Reference: 1 / 2 / 4 / 8 GCP e2-standard-8 CPU VMs, gloo over TCP (BASELINE.md).  Scaling is "
            "strong (global batch 64 split over the GPUs, ref src/train_dist.py:133), so per-GPU work shrinks "
            "to 8 images per step at N = 8.  Predicted columns: the one-GPU loopback measurement of the "
            "per-rank step (per-rank batch 64/N, exchange with N-1 virtual peers) + one xGMI hop + the "
            "pushes' link time (175 KB per peer per step at the assumed link rate); predicted "
            "time_elapsed (the reference's span: t0 after the imports): an N-rank rendezvous measured on the "
            "CPU, the N = 1 GPU bring-up, "
            "the exchange bring-up of a 2-rank rehearsal and epoch 0 at the predicted step; see the "
            "module docstring of tools/scaling_report.py."]
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
        ax.plot(*zip(*pts), "s-", color="tab:orange", label="MI355X, t0 (after imports) -> epoch 0 done")
    pts = [(r["n"], r["epoch_s"]) for r in rows if r["epoch_s"]]
    if pts:
        ax.plot(*zip(*pts), "^-", color="tab:blue", label="MI355X, warm epoch (938 steps + validation)")
    pts = [(r["n"], r["pred_epoch_s"]) for r in rows if r.get("pred_epoch_s")]
    if pts:
        ax.plot(*zip(*pts), "^--", color="tab:cyan", label="MI355X, predicted warm epoch (loopback + hop + link)")
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
    ap.add_argument("--no-predict", dest="predict", action="store_false")
    ap.add_argument("--hop-us", type=float, default=1.0, help="assumed xGMI one-way hop added for N > 1")
    ap.add_argument("--link-gbs", type=float, default=153.0,
                    help="assumed xGMI bandwidth per link and direction (GB/s) for the pushes' wire time")
    ap.add_argument("--loopback-log", help="exchange_loopback.py output replacing the built-in step table")
    ap.add_argument("--cpu-bringup", nargs="*", default=[],
                    help="bench.py --device cpu --gpus N JSON lines (spawn / import / rendezvous at N ranks)")
    ap.add_argument("--rehearsal", help="a 2-rank gloo GPU rehearsal's JSON line (exchange bring-up phases; "
                                        "run with CSED_TIME_PATHS=1 so the path selection is timed too)")
    ap.add_argument("--rccl-init", help="tools/rccl_init_probe.py output: the RCCL communicator's creation, added "
                                         "for an eager-RCCL bring-up (bench.py --eager-rccl); the default creates "
                                         "it lazily, after the span")
    a = ap.parse_args(argv)
    by_n = load_records(a.inputs)
    if not by_n:
        print("no bench records found", file=sys.stderr)
        return 1
    pred = None
    if a.predict:
        wire_us = WIRE_BYTES / (a.link_gbs * 1e3) if a.link_gbs > 0 else 0.0
        pred = predict(by_n, load_loopback(a.loopback_log) if a.loopback_log else LOOPBACK_STEP_US, a.hop_us,
                       wire_us=wire_us)
        reh = load_records([a.rehearsal]).get(2) if a.rehearsal else None
        terms: dict = {}
        for n, t in predict_time_elapsed(by_n, pred, load_records(a.cpu_bringup) if a.cpu_bringup else {},
                                         reh, load_rccl_init(a.rccl_init) if a.rccl_init else None,
                                         terms).items():
            pred[n]["time_elapsed_s"] = t
    rows = table(by_n, pred)
    out = Path(a.out)
    out.parent.mkdir(parents=True, exist_ok=True)
    md = markdown(rows, a.title)
    if pred and terms:
        md += "\nPredicted time_elapsed_s, term by term (s):\n\n| N | " + " | ".join(next(iter(terms.values()))) + " |\n"
        md += "|---:|" + "---:|" * len(next(iter(terms.values()))) + "\n"
        for n, t in sorted(terms.items()):
            md += f"| {n} | " + " | ".join(f"{v:.4f}" for v in t.values()) + " |\n"
        md += ("\nSources: hip_ctx_wait_1, setup_1 and epoch0 from the N = 1 GPU record; rendezvous_N from "
               "`bench.py --gpus N --device cpu` under torchrun (N concurrent processes: their import skew) and "
               "pg_init_N its process-group creation (gloo over N ranks: the control plane); rccl_init (only "
               "with --rccl-init: an eager RCCL bring-up) from tools/rccl_init_probe.py; exchange_bringup from the 2-rank gloo rehearsal with CSED_TIME_PATHS=1; "
               "epoch0_N at the predicted step.\n")
    out.with_suffix(".md").write_text(md)
    png = plot(rows, out.with_suffix(".png"), a.title)
    print(md)
    if png:
        print(f"wrote {out.with_suffix('.png')}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
