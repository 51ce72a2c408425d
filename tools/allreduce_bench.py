"""Latency of the 87 KB gradient all-reduce: one-shot IPC kernel vs the process group.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/allreduce_bench.py [--gloo]

With --gloo the bootstrap group is gloo and ranks may share one GPU (only the IPC
path is timed then); otherwise the group is RCCL and both paths are timed, each
as 200 calls replayed from a HIP graph (per-call time = graph time / 200).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.parallel.comm import DistContext  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.parallel.ipc import make_allreduce  # noqa: E402


def timed_graph(fn, dev, calls=200, reps=5):
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):  # (see engine/fused.py _capture)
        for _ in range(calls):
            fn()
    ts = []
    for _ in range(reps):
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize(dev)
        ts.append((time.perf_counter() - t0) / calls * 1e6)
    return sorted(ts)[len(ts) // 2]


def main():
    gloo = "--gloo" in sys.argv
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ngpu = torch.cuda.device_count()
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", rank)) % ngpu)
    torch.cuda.set_device(dev)
    be = "gloo" if gloo else "nccl"
    kw = {} if gloo else {"device_id": dev}
    dist.init_process_group(be, rank=rank, world_size=world, **kw)
    ctx = DistContext(rank, world, dev.index, dev, be)
    n = 21840
    x = torch.randn(n, device=dev)
    ar = make_allreduce(ctx, n, mode=os.environ.get("CSED_ONESHOT", "auto"))
    out = {}
    if ar is not None:
        out["ipc_us"] = timed_graph(lambda: ar(x), dev)
        out["ipc_errors"] = ar.error()
    if not gloo:
        out["rccl_us"] = timed_graph(lambda: dist.all_reduce(x), dev)
    if rank == 0:
        print(f"world={world} backend={be} n={n} fp32: " + ", ".join(f"{k}={v:.2f}" if isinstance(v, float) else
                                                               f"{k}={v}" for k, v in out.items()), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
