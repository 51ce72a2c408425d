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


def test_scaling_report_prediction_from_loopback_log(tmp_path):
    """Predicted columns: per-rank step at batch 64/N from a loopback log + the hop; the epoch
    keeps the N = 1 record's non-step remainder; measured / predicted for the records given."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import scaling_report as sr

    lb = tmp_path / "lb.log"
    lb.write_text("B= 64 N=1 update 5.87 us  step  15.00 us  stamps ...\n"
                  "B= 32 N=2 update 6.24 us  step  16.00 us\nB= 16 N=4 update 6.39 us  step  16.50 us\n"
                  "B=  8 N=8 update 6.81 us  step  17.00 us  comm_errors 0\nnoise\n")
    steps = sr.load_loopback(lb)
    assert steps == {(64, 1): 15.0, (32, 2): 16.0, (16, 4): 16.5, (8, 8): 17.0}
    by_n = {1: {"n_gpus": 1, "value": 64 / 15e-6, "ms_per_step": 0.015, "epoch_s": 938 * 15e-6 + 0.002}}
    pred = sr.predict(by_n, steps, hop_us=1.0)
    assert abs(pred[1]["step_us"] - 15.0) < 1e-9 and abs(pred[8]["step_us"] - 18.0) < 1e-9
    assert abs(pred[8]["epoch_s"] - (938 * 18e-6 + 0.002)) < 1e-9
    assert abs(pred[2]["images_s"] - 64 / 17e-6) < 1e-3
    rows = sr.table(by_n, pred)
    assert [r["n"] for r in rows] == [1, 2, 4, 8] and abs(rows[0]["vs_pred"] - 1.0) < 1e-9
    assert rows[3]["vs_pred"] is None  # no N = 8 record yet: prediction only
    md = sr.markdown(rows, "t")
    assert "predicted epoch s" in md
    # the pushes' link time adds to every N > 1
    pw = sr.predict(by_n, steps, hop_us=1.0, wire_us=1.5)
    assert abs(pw[8]["step_us"] - 19.5) < 1e-9 and abs(pw[1]["step_us"] - 15.0) < 1e-9
    assert abs(sr.WIRE_BYTES / (153.0 * 1e3) - 1.142) < 1e-3
    # the built-in table covers every N of the strong-scaling curve
    assert all(n in sr.predict({}, sr.LOOPBACK_STEP_US, 1.0) for n in (1, 2, 4, 8))


def test_scaling_report_predicts_time_elapsed():
    """Predicted time_elapsed (round-6 model): max(HIP-context wait, N-rank rendezvous) + the RCCL
    communicator's creation (N > 1), the N = 1 GPU set-up, the exchange bring-up of a 2-rank
    rehearsal (N > 1) and epoch 0 at the predicted step -- each term from a record."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import scaling_report as sr

    ph1 = {"spawn": 0.0, "import_torch": 1.4, "import_pkg": 0.01, "process_group": 0.2, "data_wait": 0.1,
           "engine": 0.05, "capture": 0.2, "test_upload": 0.01}
    by_n = {1: {"n_gpus": 1, "value": 1.0, "ms_per_step": 0.014, "epoch_s": 0.013, "epoch0_s": 0.05,
                "bringup_s": ph1}}
    steps = {(64, 1): 14.0, (8, 8): 13.0, (32, 2): 13.5}
    pred = sr.predict(by_n, steps, hop_us=1.0)
    cpu = {2: {"n_gpus": 2, "bringup_s": {"rendezvous": 0.1, "process_group": 0.12}},
           8: {"n_gpus": 8, "bringup_s": {"rendezvous": 0.3, "process_group": 0.35}}}
    reh = {"n_gpus": 2, "bringup_s": {"engine.ipc_open": 0.02, "engine.self_test": 0.03, "engine.path_timing": 0.01}}
    rccl = {"init_process_group_s": 0.04, "first_broadcast_s": 0.01}
    terms = {}
    te = sr.predict_time_elapsed(by_n, pred, cpu, reh, rccl, terms)
    base = 0.1 + 0.05 + 0.2 + 0.01
    assert abs(te[1] - (0.2 + base + 0.05)) < 1e-9
    # N = 2: rendezvous + process group (0.1 + 0.02) hide under the context wait, then the RCCL
    # term; N = 8: they are longer (0.3 + 0.05)
    assert abs(te[2] - (0.2 + 0.05 + base + 0.06 + 0.05 + 938 * 0.5e-6)) < 1e-9
    assert abs(te[8] - (0.35 + 0.05 + base + 0.06 + 0.05)) < 1e-9  # step_8 = 13 + 1 hop = step_1
    assert set(terms) == {1, 2, 8} and abs(terms[8]["total"] - te[8]) < 1e-12
    assert sr.predict_time_elapsed({}, pred, cpu, reh) == {}
