"""Debug helper: compare the local and the (world-1) all-reduce step paths of the fused engine."""
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402


def main():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    data = synthetic_mnist(2048, seed=2)
    order = torch.randperm(2048)
    for staged in (True, False):
        for spg, n in ((8, 20), (1, 3), (4, 4)):
            res = []
            for comm in (False, True):
                torch.manual_seed(1)
                e = FusedLeNetTrainer(Net().to(dev), data, lr=0.02, momentum=0.5, global_batch=64, comm=comm)
                e.staged = staged and e.staged
                e.set_epoch_order(order)
                e.run_steps(n, steps_per_graph=spg)
                torch.cuda.synchronize()
                res.append((e.flat.data.clone(), e.xstage.clone(), e.cursor.item(), e.step_count.item()))
            a, b = res
            print(f"staged={staged} spg={spg} n={n}: params {torch.equal(a[0], b[0])} "
                  f"xstage {torch.equal(a[1], b[1])} cursor {a[2]} {b[2]} step {a[3]} {b[3]}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
