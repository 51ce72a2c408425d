"""tools/scaling_report.py: bench JSON lines at N = 1/2/4/8 -> table + chart (CPU)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_scaling_report_from_bench_lines_and_scale_json(tmp_path):
    lines = []
    for n, ms in ((1, 0.0161), (2, 0.019), (4, 0.0195), (8, 0.021)):
        lines.append(json.dumps({"metric": "m", "n_gpus": n, "value": 64 / (ms * 1e-3), "ms_per_step": ms,
                                 "epoch_s": 938 * ms * 1e-3, "time_elapsed_s": 2.5, "dtype": "bf16",
                                 "config": {"allreduce": "fused-ipc" if n > 1 else "none"}}))
    logf = tmp_path / "bench.log"
    logf.write_text("noise\n" + "\n".join(lines[:2]) + "\n")
    scale = tmp_path / "SCALE.json"  # driver-style document: records nested anywhere
    scale.write_text(json.dumps({"runs": [{"n": 4, "result": json.loads(lines[2])},
                                          {"n": 8, "result": json.loads(lines[3])}]}))
    out = tmp_path / "rep" / "scaling"
    r = subprocess.run([sys.executable, "tools/scaling_report.py", str(logf), str(scale), "--out", str(out)],
                       cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    md = (tmp_path / "rep" / "scaling.md").read_text()
    rows = [l for l in md.splitlines() if l.startswith("| ") and l[2].isdigit()]
    assert [int(l.split("|")[1]) for l in rows] == [1, 2, 4, 8]
    assert "17.53" in md and "5.00" in md  # the reference's curve alongside
    assert "100.0%" in rows[0]  # N = 1 efficiency
    assert (tmp_path / "rep" / "scaling.png").stat().st_size > 1000
