"""Print a one-screen summary of a GPU iteration's logs: python tools/summarize_iter.py TAG
(gpurun_out/TAG_tests.log, TAG_*stages.log, TAG_bench*.log)."""
import glob
import json
import os
import sys

tag = sys.argv[1]
d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
t = os.path.join(d, f"{tag}_tests.log")
if os.path.exists(t):
    lines = [l.strip() for l in open(t) if l.strip()]
    print("tests:", lines[-1] if lines else "(empty)")
    for l in lines:
        if l.startswith("FAILED") or " FAILED " in l:
            print("  ", l)
for f in sorted(glob.glob(os.path.join(d, f"{tag}_*stages.log"))):
    for l in open(f):
        if "kernel" in l or "realtime" in l or "first tile" in l:
            print(os.path.basename(f), l.rstrip())
for f in sorted(glob.glob(os.path.join(d, f"{tag}_bench*.log"))):
    for l in open(f):
        if l.startswith("{"):
            r = json.loads(l)
            print(f"{os.path.basename(f):28s} {1e3 * r['ms_per_step']:8.2f} us/step {r['value'] / 1e6:8.2f} M img/s "
                  f"t_el {r.get('time_elapsed_s')} epoch {r.get('epoch_s')} val_acc {r.get('val_acc')}")
