"""Multi-process data parallelism on CPU (gloo): DDP reducer parity, bucketing, trainers, P2P."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ddp_worker(rank, world, port, q, bucket_mb):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.nn.functional as F

    from csed_514_project_distributed_training_using_pytorch_amd.models import Net
    from csed_514_project_distributed_training_using_pytorch_amd.optim import FusedSGD
    from csed_514_project_distributed_training_using_pytorch_amd.parallel import DDP, destroy, init_distributed

    ctx = init_distributed(rank=rank, world_size=world, backend="gloo", device="cpu")
    torch.manual_seed(100 + rank)  # different init per rank: DDP must broadcast rank 0's
    net = Net().eval()
    ddp = DDP(net, bucket_cap_mb=bucket_mb)
    opt = FusedSGD(net.parameters(), lr=0.05, momentum=0.5, flat=ddp.flat)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(8 * world, 1, 28, 28, generator=g)
    t = torch.randint(0, 10, (8 * world,), generator=g)
    xs, ts = x[rank * 8:(rank + 1) * 8], t[rank * 8:(rank + 1) * 8]
    init = ddp.flat.data.clone()
    for _ in range(3):
        opt.zero_grad()
        F.nll_loss(ddp(xs), ts).backward()
        opt.step()
    q.put((rank, init.numpy().copy(), ddp.flat.data.numpy().copy(), ddp.bucket_sizes_bytes()))
    destroy()


@pytest.mark.parametrize("world,bucket_mb", [(2, 25.0), (2, 0.02), (4, 0.02), (8, 0.02)])
def test_ddp_matches_single_process_full_batch(world, bucket_mb):
    import torch.nn.functional as F

    from csed_514_project_distributed_training_using_pytorch_amd.models import Net
    from csed_514_project_distributed_training_using_pytorch_amd.optim import FusedSGD

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, world, port, q, bucket_mb)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # replicas start identical (rank 0 broadcast) and stay bitwise identical
    res = [(r, torch.from_numpy(a), torch.from_numpy(b), c) for r, a, b, c in res]
    for r in res[1:]:
        assert torch.equal(res[0][1], r[1])
        assert torch.equal(res[0][2], r[2])
    if bucket_mb < 1:
        assert len(res[0][3]) >= 2  # several buckets -> overlap with backward
    # reference: one process, full batch of 8 * world, same init
    net = Net().eval()
    torch.manual_seed(100)
    ref = Net().eval()
    opt = FusedSGD(ref.parameters(), lr=0.05, momentum=0.5)
    opt.flat.data.copy_(res[0][1])
    g = torch.Generator().manual_seed(7)
    x = torch.randn(8 * world, 1, 28, 28, generator=g)
    t = torch.randint(0, 10, (8 * world,), generator=g)
    for _ in range(3):
        opt.zero_grad()
        F.nll_loss(ref(x), t).backward()
        opt.step()
    torch.testing.assert_close(res[0][2], opt.flat.data, rtol=1e-5, atol=1e-6)


def test_plan_buckets():
    from csed_514_project_distributed_training_using_pytorch_amd.parallel.ddp import plan_buckets

    numels = [250, 10, 5000, 20, 16000, 50, 500, 10]
    assert plan_buckets(numels, 10 ** 9) == [list(range(8))]
    b = plan_buckets(numels, 16560)
    assert b == [[4, 5, 6, 7], [0, 1, 2, 3]]  # FC bucket first (ready first in backward), then conv
    assert plan_buckets([100], 10) == [[0]]


def _run(cmd, timeout=300, env=None):
    e = dict(os.environ)
    e.update(env or {})
    e.setdefault("CSED_AUTOBUILD", "0")
    return subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=e)


def test_single_process_cli_cpu(tmp_path):
    r = _run([sys.executable, "src/train.py", "--device", "cpu", "--synthetic", "--epochs", "1", "--train-size",
              "640", "--test-size", "200", "--out-dir", str(tmp_path)])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Train Epoch: 1 [0/640 (0%)]\tLoss: " in r.stdout
    assert "Test set: Avg. loss: " in r.stdout and "time_elapsed=" in r.stdout
    assert (tmp_path / "results" / "model.pth").exists() and (tmp_path / "results" / "optimizer.pth").exists()
    sd = torch.load(tmp_path / "results" / "model.pth", weights_only=True)
    assert list(sd.keys())[0] == "conv1.weight" and len(sd) == 8
    assert (tmp_path / "images" / "train_test_curve.png").exists()


def test_distributed_cli_cpu_two_ranks(tmp_path):
    r = _run([sys.executable, "-m", "csed_514_project_distributed_training_using_pytorch_amd.parallel.launch",
              "--nproc", "2", "--timeout", "240", "src/train_dist.py", "--device", "cpu", "--synthetic",
              "--epochs", "2", "--train-size", "512", "--test-size", "200", "--engine", "modular",
              "--out-dir", str(tmp_path), "--bucket-mb", "0.02", "--check-replicas", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("Epoch=")]
    assert len(lines) == 4  # 2 epochs x 2 ranks print (every VM printed in the reference)
    assert "time_elapsed=" in lines[0]
    # the per-epoch cross-rank parameter hash ran and found identical replicas
    assert r.stdout.count("parameters bitwise identical on 2 ranks") == 2
    sd = torch.load(tmp_path / "model.pt", weights_only=True)
    assert "conv1.weight" in sd and not any(k.startswith("module.") for k in sd)


def test_p2p_smoke_two_ranks():
    port = str(_port())
    env = {"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": port}
    p0 = subprocess.Popen([sys.executable, "src/run1.py"], cwd=ROOT, stdout=subprocess.PIPE, text=True,
                          env={**os.environ, **env})
    p1 = subprocess.Popen([sys.executable, "src/run2.py"], cwd=ROOT, stdout=subprocess.PIPE, text=True,
                          env={**os.environ, **env})
    o0, _ = p0.communicate(timeout=120)
    o1, _ = p1.communicate(timeout=120)
    assert p0.returncode == 0 and p1.returncode == 0
    assert "Rank  0  has data  tensor(1.)" in o0
    assert "Rank  1  has data  tensor(1.)" in o1


def test_bench_self_spawns_ranks_cpu():
    """bench.py --gpus N without a torchrun environment starts N ranks itself (one per GPU;
    here gloo on the CPU) and rank 0 prints exactly one JSON line whose n_gpus is the
    process group's size."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--backend", "gloo", "--device", "cpu",
                        "--steps", "3", "--warmup", "1"], cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    js = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(js) == 1, r.stdout
    import json

    rec = json.loads(js[0])
    assert rec["n_gpus"] == 2 and rec["config"]["process_group"] == {"backend": "gloo", "ranks": 2}
    assert rec["config"]["parallelism"] == "dp2" and rec["steps"] == 3 and rec["value"] > 0
    assert rec["time_elapsed_s"] > 0
    # every rank's data-parallel diagnostics, every key present (a failing N-GPU bring-up names
    # its stage: peer access, IPC open, self-test, path timing, error word, first mismatch)
    from csed_514_project_distributed_training_using_pytorch_amd.parallel.ipc import DIAG_KEYS

    diag = rec["exchange_diag"]
    assert [d["rank"] for d in diag] == [0, 1], diag
    for d in diag:
        assert set(DIAG_KEYS) <= set(d), d


def test_bench_eight_ranks_bringup_phases_cpu():
    """bench.py --gpus 8 --device cpu: the driver's 8-rank launch shape on the CPU (spawn, eight
    concurrent `import torch`, an 8-rank rendezvous).  The JSON's bringup_s carries the per-phase
    breakdown of time_elapsed_s (max over ranks) that the driver's SCALE run records."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--device", "cpu", "--steps", "2",
                        "--warmup", "1"], cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    js = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(js) == 1, r.stdout
    import json

    rec = json.loads(js[0])
    assert rec["n_gpus"] == 8 and rec["config"]["parallelism"] == "dp8"
    ph = rec["bringup_s"]
    assert {"spawn", "import_torch", "import_pkg", "process_group"} <= set(ph), ph
    assert all(v >= 0 for v in ph.values()), ph
    # every phase is a part of the span it is measured in: the imports (and the spawn) come
    # before the reference's t0, the rendezvous after it
    assert ph["process_group"] <= rec["time_elapsed_s"] + 1e-3, rec
    assert ph["spawn"] + ph["import_torch"] + ph["import_pkg"] + ph["process_group"] \
        <= rec["process_elapsed_s"] + 1e-3, rec
    assert rec["replicas_identical"] is True, rec


def test_bench_rejects_world_size_mismatch_cpu():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--device", "cpu", "--steps", "1", "--warmup",
                        "0"], cwd=ROOT, capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr



def _replica_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from csed_514_project_distributed_training_using_pytorch_amd.parallel import destroy, init_distributed
    from csed_514_project_distributed_training_using_pytorch_amd.parallel.comm import replica_checksum

    ctx = init_distributed(rank=rank, world_size=world, backend="gloo", device="cpu")
    t = torch.linspace(-1, 1, 21840)
    same = replica_checksum(ctx, t)[0]
    u = t.clone()
    if rank == 1:  # one ulp of one parameter on one replica
        u[12345] = torch.nextafter(u[12345], torch.tensor(2.0))
    diverged = replica_checksum(ctx, u)[0]
    v = t.clone()
    if rank == 1:  # two entries swapped: same multiset of bits, different positions
        v[[10, 11]] = v[[11, 10]]
    swapped = replica_checksum(ctx, v)[0]
    q.put((rank, same, diverged, swapped))
    destroy()


def test_replica_checksum_detects_divergence():
    """--check-replicas' collective: equal replicas pass; a one-ulp change or a
    swap of two parameters on one rank is caught on every rank."""
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_replica_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, same, diverged, swapped in res:
        assert same and not diverged and not swapped, (rank, same, diverged, swapped)
