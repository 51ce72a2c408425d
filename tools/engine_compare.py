"""Step time of the two GPU engines across batch sizes (one MI355X).

    python tools/engine_compare.py [B ...]

fused   = csed::lenet_train + csed::lenet_update, HIP-graph replay (bench.py's engine)
modular = per-op HIP kernels + autograd + FusedSGD, eager launches from Python
Both run SGD lr 0.02 momentum 0.5 with dropout on synthetic data, fp16 and bf16.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.data.mnist import MNIST_MEAN, MNIST_STD  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.modular import ModularTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.ops import set_compute_dtype  # noqa: E402


def fused_ms(data, B, dt, steps=20):
    torch.manual_seed(1)
    eng = FusedLeNetTrainer(Net().cuda(), data, lr=0.02, momentum=0.5, global_batch=B, compute_dtype=dt)
    eng.set_epoch_order(torch.randperm(len(data)))
    spg = max(1, min(8, eng.full_steps() // 2))
    eng.prepare(spg)
    eng.run_steps(spg, spg)
    torch.cuda.synchronize()
    n = min(steps, eng.full_steps() - spg)
    n -= n % spg
    t0 = time.perf_counter()
    eng.run_steps(n, spg)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def modular_ms(data, B, dt, steps=20):
    torch.manual_seed(1)
    set_compute_dtype(dt)
    net = Net().cuda()
    tr = ModularTrainer(net, lr=0.02, momentum=0.5)
    imgs = data.images[:B].cuda()
    x = ((imgs.float() / 255.0 - MNIST_MEAN) / MNIST_STD).view(B, 1, 28, 28)
    t = data.labels[:B].cuda()
    for _ in range(3):
        tr.train_batch(x, t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.train_batch(x, t)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    bs = [int(a) for a in sys.argv[1:]] or [64, 1024, 8192]
    data = synthetic_mnist(max(16384, 4 * max(bs)), seed=0)
    for dt in (torch.bfloat16, torch.float16):
        for B in bs:
            f = fused_ms(data, B, dt)
            m = modular_ms(data, B, dt)
            print(f"{str(dt).split('.')[-1]:9s} B={B:5d}  fused {f:8.3f} ms/step ({B / f * 1e-3:8.2f} M img/s)   "
                  f"modular {m:8.3f} ms/step ({B / m * 1e-3:8.2f} M img/s)", flush=True)


if __name__ == "__main__":
    main()
