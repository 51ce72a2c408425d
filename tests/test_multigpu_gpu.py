"""The fused gradient exchange with ONE RANK PER GPU over RCCL + xGMI (parallel/dpcheck.py),
for the driver's multi-GPU box: world = min(device_count, 8) ranks; the fused exchange must
be selected (where it also times faster than RCCL: the engine keeps the faster path), match
the CSED_ALLREDUCE=rccl run (bitwise at world 2), leave bitwise-identical replicas and raise no
error word; every pair of GPUs must report peer access.  Ref: src/train_dist.py:63,83,146.

On a one-GPU box the GPU test is skipped; its CPU plumbing (launch, rendezvous, replica
check) runs under gloo in test_dpcheck_plumbing_gloo_cpu."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MOD = "csed_514_project_distributed_training_using_pytorch_amd.parallel.dpcheck"


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(nproc: int, extra: list[str], timeout: int) -> dict:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m", MOD, *extra]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", CSED_IPC_TIMEOUT_S="10")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("DPCHECK ")]
    assert lines, f"rc {r.returncode}\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    rec = json.loads(lines[-1][len("DPCHECK "):])
    rec["_rc"] = r.returncode
    return rec


@pytest.mark.gpu
@pytest.mark.skipif(torch.cuda.device_count() < 2,
                    reason="one rank per GPU needs >= 2 GPUs (this box has fewer); CPU plumbing: "
                           "test_dpcheck_plumbing_gloo_cpu")
def test_fused_exchange_one_rank_per_gpu():
    world = min(torch.cuda.device_count(), 8)
    rec = _run(world, ["--steps", "16"], timeout=600)
    assert rec["_rc"] == 0 and rec["all_ranks_ok"], rec
    assert rec["world"] == world and rec["gpus"] == world, rec
    assert all(rec["peer_access"].values()), rec["peer_access"]
    f = rec["fused"]
    assert f["error_word"] == 0 and f["replicas_identical"], f
    # the fused exchange is kept unless it timed slower than RCCL (then the timing says so)
    if f["allreduce"] != "fused-ipc":
        t = f["path_timing_us"]
        assert t and t["kept"] == "rccl" and t["fallback_step_us"] < t["fused_step_us"], f
    elif world == 2:
        assert rec["fused_equals_rccl_bitwise"], rec
    assert rec["rccl"]["allreduce"] == "rccl" and rec["rccl"]["replicas_identical"], rec


def test_dpcheck_plumbing_gloo_cpu():
    from csed_514_project_distributed_training_using_pytorch_amd.parallel.ipc import DIAG_KEYS

    rec = _run(2, ["--device", "cpu", "--steps", "3"], timeout=300)
    assert rec["_rc"] == 0 and rec["all_ranks_ok"] and rec["replicas_identical"], rec
    assert rec["backend"] == "gloo" and rec["world"] == 2
    assert [d["rank"] for d in rec["exchange_diag"]] == [0, 1]
    assert all(set(DIAG_KEYS) <= set(d) for d in rec["exchange_diag"]), rec["exchange_diag"]


@pytest.mark.gpu
def test_dpcheck_two_ranks_shared_gpu_rehearsal():
    """The one-rank-per-GPU check's rehearsal on a one-GPU box: two gloo ranks sharing the GPU run
    dpcheck's fused (auto) and process-group paths from the same state; the DPCHECK line carries
    every rank's exchange diagnostics (peer access, IPC open, self-test, path timing, error word,
    first mismatch) and both paths agree bitwise (a + b is order-free)."""
    from csed_514_project_distributed_training_using_pytorch_amd.parallel.ipc import DIAG_KEYS

    rec = _run(2, ["--backend", "gloo", "--steps", "8"], timeout=600)
    assert rec["_rc"] == 0 and rec["all_ranks_ok"], rec
    diag = rec["fused"]["exchange_diag"]
    assert [d["rank"] for d in diag] == [0, 1] and all(set(DIAG_KEYS) <= set(d) for d in diag), diag
    assert all(d["ipc_open"] == "ok" and d["self_test"] is True and d["error_word"] == 0 for d in diag), diag
    assert rec["fused"]["allreduce"] == "fused-ipc" and rec["fused_equals_rccl_bitwise"], rec
