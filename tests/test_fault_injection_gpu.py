"""Fault injection into the fused gradient exchange (csrc/comm ipc_set_mute: a rank's pushes go to
a dead-end buffer, so to its peers it is a dead rank) and the two recovery paths that depend on
the exchange's error word:

* the kernel side: a peer wait ends at CSED_IPC_TIMEOUT_S with the error word raised, and once it
  is raised later calls never wait again (a dead peer costs one timeout, not one per step);
* ``bench.py``: a run whose exchange timed out is re-measured on the process-group path
  (``config.comm_retry``) and still prints one valid JSON line;
* ``train_dist.py`` (engine/cli.py dist_main): the epoch is rolled back and re-run on the process
  group's all-reduce, ending bitwise where a clean CSED_ALLREDUCE=rccl run ends.

The reference has only the process group's own timeout (ref src/train_dist.py:146)."""
import json
import os
import subprocess
import sys
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _engine(B, loopback_world):
    from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist
    from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer
    from csed_514_project_distributed_training_using_pytorch_amd.models import Net

    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    return FusedLeNetTrainer(Net().to(dev), synthetic_mnist(1024, seed=3), lr=0.05, momentum=0.5, global_batch=B,
                             loopback_world=loopback_world)


def test_dead_peer_times_out_once_and_releases():
    """Loopback world 2 with a dead virtual peer: the first step's waits end at the 0.3 s bound
    with the error word set; the next steps poll once and do not wait again; close() releases
    the IPC buffers (the id is retired)."""
    eng = _engine(8, 2)
    eng.exch_timeout_s = 0.3
    eng.set_epoch_order(torch.randperm(1024, generator=torch.Generator().manual_seed(0)))
    eng.step()  # a healthy step first: no error
    torch.cuda.synchronize()
    assert eng.comm_errors() == 0
    eng.inject_exchange_fault()
    t0 = time.perf_counter()
    eng.step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    assert eng.comm_errors() != 0
    assert 0.25 < t1 - t0 < 2.0, t1 - t0  # one bounded wait, not a hang
    for _ in range(6):  # the error word is set: no more waiting
        eng.step()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    assert t2 - t1 < 0.25, t2 - t1
    xid = eng.exch.id
    eng.close()
    assert eng.exch is None
    with pytest.raises(RuntimeError):
        torch.ops.csed.ipc_error(xid, False)


def test_bench_remeasures_after_injected_fault(tmp_path):
    """bench.py with a dead virtual peer: the first run's exchange times out, the bench releases
    the IPC buffers and re-measures without the exchange; one valid JSON line with
    config.comm_retry, and no comm_error in the reported (second) run."""
    env = dict(os.environ, CSED_IPC_TIMEOUT_S="0.1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--global-batch", "8", "--loopback-world", "2",
           "--inject-exchange-fault", "--steps", "50", "--warmup", "5", "--no-epoch"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=tmp_path)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert "comm_retry" in rec["config"], rec
    assert "loopback2" in rec["config"]["comm_retry"], rec
    assert "comm_error" not in rec, rec
    assert rec["config"]["allreduce"] == "none", rec
    assert rec["value"] > 0 and rec["steps"] == 50
    assert any(k.startswith("retry.") for k in rec["bringup_s"]), rec["bringup_s"]


def _dist_run(out, extra, env_extra):
    env = dict(os.environ, CSED_IPC_TIMEOUT_S="0.2", **env_extra)
    cmd = [sys.executable, "-m", "csed_514_project_distributed_training_using_pytorch_amd.parallel.launch",
           "--nproc", "2", os.path.join(ROOT, "src", "train_dist.py"), "--backend", "gloo", "--epochs", "2",
           "--batch-size", "16", "--synthetic", "--train-size", "2048", "--test-size", "1000", "--no-plot",
           "--out-dir", str(out), *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r, torch.load(os.path.join(out, "model.pt"), weights_only=True)


def test_dist_epoch_rerun_after_injected_fault_matches_clean_run(tmp_path):
    """Two gloo ranks on the shared GPU, fused exchange: the last rank goes dead in epoch 0, the
    epoch is detected, rolled back and re-run on the process group's all-reduce (then epoch 1
    too); the final model equals, bit for bit, a run that used the process group's all-reduce
    from the start (CSED_ALLREDUCE=rccl)."""
    r_fault, sd_fault = _dist_run(tmp_path / "fault", ["--inject-exchange-fault", "0"], {})
    assert "re-running the epoch on the process-group all-reduce" in r_fault.stderr, r_fault.stderr[-3000:]
    r_clean, sd_clean = _dist_run(tmp_path / "clean", [], {"CSED_ALLREDUCE": "rccl"})
    assert "re-running" not in r_clean.stderr
    assert sd_fault.keys() == sd_clean.keys()
    for k in sd_clean:
        assert torch.equal(sd_fault[k], sd_clean[k]), k
    # and the epoch lines: two epochs per rank in each run, the faulted epoch printed once
    for r in (r_fault, r_clean):
        assert r.stdout.count("Epoch=") == 2 * 2, r.stdout  # (two ranks' lines may share a line)


@pytest.mark.parametrize("stage", ["open", "selftest"])
def test_bench_two_ranks_rejected_exchange_still_reports(tmp_path, stage):
    """bench.py --gpus 2 (two gloo ranks sharing the GPU) with the fused exchange rejected on the
    last rank (CSED_TEST_EXCH_REJECT: a failed buffer mapping / self-test): every rank falls back to
    the process group's all-reduce, the line still carries a valid value, and exchange_diag names
    the failing stage on the failing rank (the first-run diagnostics of a real N-GPU node)."""
    from csed_514_project_distributed_training_using_pytorch_amd.parallel.ipc import DIAG_KEYS

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(CSED_TEST_EXCH_REJECT=stage, CSED_IPC_TIMEOUT_S="2")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--steps", "20",
           "--warmup", "2", "--no-epoch", "--no-fp32-record"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=tmp_path)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["value"] and rec["value"] > 0 and rec["replicas_identical"] is True, rec
    assert rec["config"]["allreduce"] == "rccl", rec  # (the process-group path: gloo here)
    diag = rec["exchange_diag"]
    assert [d["rank"] for d in diag] == [0, 1] and all(set(DIAG_KEYS) <= set(d) for d in diag), diag
    assert all(d["allreduce"] == "rccl" and d["ranks_per_gpu"] == 2 for d in diag), diag
    if stage == "open":
        assert all(d["ipc_open"] != "ok" and d["self_test"] is None for d in diag), diag
    else:
        assert all(d["ipc_open"] == "ok" for d in diag), diag
        assert diag[0]["self_test"] is True and diag[1]["self_test"] is False, diag


def test_bench_two_ranks_lazy_rccl_shared_gpu(tmp_path):
    """bench.py --gpus 2 with the default (RCCL) backend on the one GPU: the communicator is created
    lazily and the bring-up's host collectives run on the gloo control plane, so two ranks sharing a
    GPU (which RCCL itself refuses) train the fused exchange end to end -- the real N-GPU flow short
    of xGMI: a valid value, bitwise replicas, no error word, the fp32 sub-record on the reused
    exchange."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(CSED_IPC_TIMEOUT_S="5")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20", "--warmup", "2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=tmp_path)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["config"]["process_group"] == {"backend": "nccl", "ranks": 2}, rec["config"]
    assert rec["config"]["allreduce"] == "fused-ipc" and rec["value"] > 0, rec
    assert rec["replicas_identical"] is True and "comm_error" not in rec, rec
    assert all(d["error_word"] == 0 and d["self_test"] is True for d in rec["exchange_diag"]), rec["exchange_diag"]
    assert rec["fp32"]["replicas_identical"] and "fused-ipc" in rec["fp32"]["engine"], rec["fp32"]
