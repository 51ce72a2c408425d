"""GPU end-to-end: RCCL inside HIP-graph capture, CLIs on the GPU, modular engine training."""
import os
import socket
import subprocess
import sys

import pytest
import torch

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer
from csed_514_project_distributed_training_using_pytorch_amd.models import Net

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_allreduce_path_inside_graph_matches_local():
    """World size 1 process group on RCCL: the reduce-only -> all_reduce -> SGD path,
    captured in a HIP graph, must give bit-identical weights to the local path."""
    import torch.distributed as dist

    from csed_514_project_distributed_training_using_pytorch_amd.parallel.comm import init_distributed

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_port())
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if not dist.is_initialized():
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        data = synthetic_mnist(2048, seed=2)
        order = torch.randperm(2048)
        res = []
        for comm in (False, True):
            torch.manual_seed(1)
            eng = FusedLeNetTrainer(Net().to(dev), data, lr=0.02, momentum=0.5, global_batch=64, comm=comm)
            eng.set_epoch_order(order)
            eng.run_steps(20, steps_per_graph=8)
            torch.cuda.synchronize()
            assert eng.capture_comm_ok is True
            res.append(eng.flat.data.clone())
        assert torch.equal(res[0], res[1])
    finally:
        dist.destroy_process_group()


def _run(args, timeout=600):
    env = dict(os.environ)
    env.setdefault("CSED_AUTOBUILD", "0")
    return subprocess.run([sys.executable, *args], cwd=ROOT, capture_output=True, text=True, timeout=timeout,
                          env=env)


@pytest.mark.parametrize("engine", ["fused", "modular"])
def test_train_cli_on_gpu(tmp_path, engine):
    r = _run(["src/train.py", "--synthetic", "--epochs", "2", "--train-size", "19200", "--test-size", "1000",
              "--engine", engine, "--out-dir", str(tmp_path)])
    assert r.returncode == 0, r.stderr[-3000:]
    losses = [float(l.split("Avg. loss: ")[1].split(",")[0]) for l in r.stdout.splitlines() if "Avg. loss" in l]
    # the synthetic set is deliberately hard (86 % after a full 60k epoch on the CPU reference)
    assert len(losses) == 3 and losses[-1] < 0.6 * losses[0], r.stdout[-2000:]
    sd = torch.load(tmp_path / "results" / "model.pth", weights_only=True)
    assert len(sd) == 8 and sd["fc2.bias"].shape == (10,)
    osd = torch.load(tmp_path / "results" / "optimizer.pth", weights_only=True)
    assert len(osd["state"]) == 8 and "momentum_buffer" in osd["state"][0]


def test_train_dist_cli_single_gpu_rank(tmp_path):
    r = _run(["-m", "csed_514_project_distributed_training_using_pytorch_amd.parallel.launch", "--nproc", "1",
              "src/train_dist.py", "--synthetic", "--epochs", "2", "--train-size", "6400", "--test-size", "1000",
              "--out-dir", str(tmp_path)])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("Epoch=")]
    assert len(lines) == 2
    assert (tmp_path / "model.pt").exists()


def test_bench_contract_json():
    """bench.py prints exactly one JSON line with the driver's fields (short run)."""
    import json

    r = _run(["bench.py", "--steps", "40", "--warmup", "8", "--steps-per-graph", "8", "--no-epoch"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip().startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in rec, k
    assert rec["n_gpus"] == 1 and rec["steps"] == 40 and rec["warmup"] == 8 and rec["dtype"] == "bf16"
    assert rec["config"]["global_batch"] == 64 and rec["value"] > 0 and rec["higher_is_better"] is True
    assert abs(rec["value"] - 64 / (rec["ms_per_step"] * 1e-3)) / rec["value"] < 0.01


def test_graft_smoke_entry():
    r = _run(["-c", "import __graft_entry__ as g; g.smoke()"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert "smoke ok" in r.stdout

