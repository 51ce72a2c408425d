"""Point-to-point connectivity smoke test shared by run1.py / run2.py (ref src/run1.py:8-37).

Rank 0 adds 1 to a zeros(1) tensor and sends it to rank 1, which receives it; both
print `Rank  r  has data  tensor(...)`.  Rendezvous: MASTER_ADDR (default 127.0.0.1),
MASTER_PORT (default 29500).  Backend gloo on CPU tensors (the reference), or
--backend nccl --device cuda to exercise RCCL between two GPUs.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(rank: int, size: int, backend: str, device: str) -> int:
    from csed_514_project_distributed_training_using_pytorch_amd.parallel.comm import destroy, init_distributed, p2p_exchange

    ctx = init_distributed(rank=rank, world_size=size, local_rank=rank, backend=backend, device=device)
    t = p2p_exchange(ctx, src=0, dst=1)
    print("Rank ", rank, " has data ", t[0].cpu(), flush=True)
    destroy()
    return 0


def main(default_rank: int, argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, default=default_rank)
    ap.add_argument("--world-size", type=int, default=2)
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--device", default="cpu")
    a = ap.parse_args(argv)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    # the reference spawns a child process per machine (mp.set_start_method("spawn"))
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    p = ctx.Process(target=run, args=(a.rank, a.world_size, a.backend, a.device))
    p.start()
    p.join()
    return p.exitcode or 0
