#!/usr/bin/env python3
"""Where the bench's bring-up goes, from a rocprofv3 HIP-API + kernel + memory-copy trace
(``tools/gpu.sh bringtrace``): every HIP call / kernel / copy longer than --min-ms, in time
order, relative to the first traced HIP call, plus the longest ones.

    python tools/bringup_trace.py <rocprofv3 output dir> [--min-ms 0.5]"""
import argparse
import csv
import glob
import os


def rows(path):
    with open(path, newline="") as f:
        yield from csv.DictReader(f)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-ms", type=float, default=0.5)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    ev = []
    for kind, pat in (("api", "*hip_api_trace.csv"), ("kernel", "*kernel_trace.csv"), ("copy", "*memory_copy_trace.csv")):
        for p in glob.glob(os.path.join(a.dir, "**", pat), recursive=True):
            for r in rows(p):
                name = r.get("Function") or r.get("Kernel_Name") or r.get("Operation") or "?"
                try:
                    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                except (KeyError, ValueError):
                    continue
                tid = r.get("Thread_Id", "")
                ev.append((s, e, kind, name[:90], tid))
    if not ev:
        print("no trace rows found under", a.dir)
        return 1
    ev.sort()
    t0 = ev[0][0]
    print(f"{len(ev)} events; span {(ev[-1][1] - t0) / 1e6:.1f} ms")
    print(f"\n-- events >= {a.min_ms} ms, in order (start ms, duration ms, kind, thread, name)")
    firsts = set()
    for s, e, k, n, tid in ev:
        d = (e - s) / 1e6
        first = (k, n) not in firsts
        firsts.add((k, n))
        if d >= a.min_ms or (k == "kernel" and first):
            print(f"{(s - t0) / 1e6:9.2f} {d:8.3f}  {k:6s} {tid:>8s} {'*' if first else ' '} {n}")
    print(f"\n-- top {a.top} by duration")
    for s, e, k, n, tid in sorted(ev, key=lambda x: x[0] - x[1])[: a.top]:
        print(f"{(s - t0) / 1e6:9.2f} {(e - s) / 1e6:8.3f}  {k:6s} {tid:>8s} {n}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
