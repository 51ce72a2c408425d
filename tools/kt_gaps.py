"""Kernel durations and inter-kernel gaps of a rocprofv3 --kernel-trace CSV (csed kernels only).
usage: python tools/kt_gaps.py <kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "csed" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[len(rows) // 3:]  # skip warm-up
dur = defaultdict(list)
gap = defaultdict(list)
for prev, cur in zip(rows, rows[1:]):
    gap[(prev["Kernel_Name"][:40], cur["Kernel_Name"][:40])].append(int(cur["Start_Timestamp"]) - int(prev["End_Timestamp"]))
for r in rows:
    dur[r["Kernel_Name"][:60]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
med = lambda xs: sorted(xs)[len(xs) // 2] / 1000
for k, v in dur.items():
    print(f"duration  {k:60s} n={len(v):4d} median {med(v):7.2f} us")
for k, v in gap.items():
    print(f"gap  {k[0]:40s} -> {k[1]:40s} n={len(v):4d} median {med(v):6.2f} us")
