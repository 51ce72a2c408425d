"""Summarise a rocprofv3 kernel trace (rocpd SQLite .db or kernel_trace.csv) as markdown.

Usage: python tools/rocpd_summary.py <run_results.db | run_kernel_trace.csv> [title]

Prints, per kernel name: launches, median / min / p95 duration (us) and the
share of total GPU kernel time -- the table committed under profiles/.
"""
import csv
import sqlite3
import statistics
import sys
from collections import defaultdict


def load(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        return [(n, (e - s) / 1000.0) for n, s, e in c.execute("select name, start, end from kernels order by start")]
    rows = list(csv.DictReader(open(path)))
    return [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0) for r in rows]


def main():
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else path
    by = defaultdict(list)
    for n, d in load(path):
        by[n].append(d)
    total = sum(sum(v) for v in by.values())
    print(f"### {title}\n")
    print("| kernel | launches | median us | min us | p95 us | share |")
    print("|---|---:|---:|---:|---:|---:|")
    for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        p95 = v[min(len(v) - 1, int(0.95 * len(v)))]
        short = n if len(n) <= 70 else n[:67] + "..."
        print(f"| `{short}` | {len(v)} | {statistics.median(v):.2f} | {v[0]:.2f} | {p95:.2f} | "
              f"{100 * sum(v) / total:.1f}% |")


if __name__ == "__main__":
    main()
