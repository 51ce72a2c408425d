"""bench.py's time spans (CPU): ``time_elapsed_s`` is the reference's span -- t0 right after
``import torch`` and the package (ref src/train_dist.py:1-11 imports, :119 t0) -- and no job
work (the synthetic-data generator, the HIP-context thread) starts before t0;
``process_elapsed_s`` keeps the span from process start."""
import importlib.util
import json
import os
import subprocess
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench_module():
    spec = importlib.util.spec_from_file_location("_bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bringup_starts_no_job_work_before_t0(monkeypatch):
    bench = _bench_module()
    calls = []
    monkeypatch.setattr(bench, "start_native_data", lambda: calls.append(("native_data", time.time())) or None)
    monkeypatch.setattr(bench, "start_gpu_context",
                        lambda phases=None, **kw: calls.append(("hip_ctx_thread", time.time())) or None)
    phases = {}
    t0, native_job, ctx_job = bench.bringup(types.SimpleNamespace(device="cuda"), phases)
    # the imports are timed and come first
    assert "import_torch" in phases and "import_pkg" in phases
    assert "torch" in sys.modules
    # both pieces of job work were started, and only after t0
    assert [c[0] for c in calls] == ["native_data", "hip_ctx_thread"]
    assert all(t >= t0 for _, t in calls)
    names = [e[0] for e in bench.BRINGUP_EVENTS]
    assert names[0] == "t0" and set(names[1:]) == {"native_data", "hip_ctx_thread"}


def test_bench_json_reports_both_spans_cpu():
    r = subprocess.run([sys.executable, "bench.py", "--device", "cpu", "--steps", "2", "--warmup", "1"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert 0 < rec["time_elapsed_s"] < rec["process_elapsed_s"]
    # the imports are outside the reference span and inside the process span
    b = rec["bringup_s"]
    assert rec["process_elapsed_s"] - rec["time_elapsed_s"] >= 0.9 * (b["import_torch"] + b["import_pkg"])
