"""Large-batch step time: the per-op (modular) engine vs the fused two-kernel step.

    python tools/large_batch_probe.py [B ...]

For each per-rank batch B: ms per training step (forward, backward, SGD) of
engine/modular.py's ModularTrainer (per-op HIP kernels + autograd, eager launches)
and of engine/fused.py's FusedLeNetTrainer (graph-replayed), fp16, synthetic data.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd import ops  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.data.mnist import MNIST_MEAN, MNIST_STD  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.modular import ModularTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402


def modular_ms(B, data, dev, iters=20):
    ops.set_compute_dtype(torch.float16)
    torch.manual_seed(1)
    net = Net().to(dev)
    tr = ModularTrainer(net, lr=0.02, momentum=0.5)
    x = ((data.images[:B].to(dev).float() / 255.0 - MNIST_MEAN) / MNIST_STD).unsqueeze(1).to(torch.float16)
    t = data.labels[:B].to(dev)
    for _ in range(3):
        tr.train_batch(x, t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        tr.train_batch(x, t)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / iters


def fused_ms(B, data, dev, steps=8):
    torch.manual_seed(1)
    eng = FusedLeNetTrainer(Net().to(dev), data, lr=0.02, momentum=0.5, global_batch=B,
                            compute_dtype=torch.float16)
    eng.set_epoch_order(torch.randperm(len(data)))
    eng.run_steps(steps, steps_per_graph=steps)
    torch.cuda.synchronize()
    eng.set_epoch_order(torch.randperm(len(data)))
    t0 = time.perf_counter()
    eng.run_steps(steps, steps_per_graph=steps)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps


def main():
    bs = [int(a) for a in sys.argv[1:]] or [1024, 8192]
    dev = torch.device("cuda")
    data = synthetic_mnist(max(bs) * 9, seed=3)
    for B in bs:
        m = modular_ms(B, data, dev)
        f = fused_ms(B, data, dev)
        print(f"B={B:6d}  modular {m:8.3f} ms ({B / m / 1e3:7.2f} M img/s)   fused {f:8.3f} ms "
              f"({B / f / 1e3:7.2f} M img/s)", flush=True)


if __name__ == "__main__":
    main()
