#!/usr/bin/env python3
"""Same-box A/B of `import torch` with and without a concurrent HIP-context thread (the round-4
bench started the context while torch imported; round 5 starts it after the reference's t0).

Each sample is a fresh child process (page cache warm after the first), alternating
A = plain `import torch` and B = the same with bench.py's context thread (ctypes hipSetDevice +
hipFree(0) on the HIP runtime torch links) started before it.  Prints one JSON line per sample
and the medians.

    python tools/import_probe.py [--n 5]
"""
from __future__ import annotations

import argparse
import json
import statistics
import subprocess
import sys

CHILD = r'''
import ctypes, importlib.util, json, os, sys, threading, time
with_ctx = sys.argv[1] == "B"
t0 = time.time()
th = None
if with_ctx:
    spec = importlib.util.find_spec("torch")
    hip = ctypes.CDLL(os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so"))
    box = {}
    def run():
        t = time.time()
        if hip.hipSetDevice(0) == 0:
            hip.hipFree(ctypes.c_void_p(0))
        box["ctx"] = time.time() - t
    th = threading.Thread(target=run, daemon=True)
    th.start()
t1 = time.time()
import torch
t2 = time.time()
if th is not None:
    th.join()
print(json.dumps({"variant": sys.argv[1], "import_torch_s": t2 - t1, "ctx_thread_s": box.get("ctx") if with_ctx else None,
                  "total_s": time.time() - t0}))
'''


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=5)
    a = ap.parse_args()
    res = {"A": [], "B": []}
    for i in range(a.n):
        for v in ("A", "B"):
            out = subprocess.run([sys.executable, "-c", CHILD, v], capture_output=True, text=True, timeout=300)
            line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
            if not line:
                print(json.dumps({"variant": v, "error": out.stderr[-500:]}))
                continue
            rec = json.loads(line[-1])
            rec["sample"] = i
            print(json.dumps(rec), flush=True)
            res[v].append(rec["import_torch_s"])
    print(json.dumps({"median_import_s": {k: statistics.median(v) if v else None for k, v in res.items()},
                      "note": "A = import torch alone, B = with the HIP-context thread running alongside"}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
