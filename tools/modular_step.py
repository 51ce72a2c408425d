"""Run N modular-engine training steps at batch B (for rocprofv3 kernel traces).

    rocprofv3 --kernel-trace --stats --output-format csv -d OUT -o run -- python3 tools/modular_step.py B N
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.data.mnist import MNIST_MEAN, MNIST_STD  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.modular import ModularTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.ops import set_compute_dtype  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    set_compute_dtype(torch.float16)
    torch.manual_seed(1)
    data = synthetic_mnist(B, seed=0)
    tr = ModularTrainer(Net().cuda(), lr=0.02, momentum=0.5)
    x = ((data.images.cuda().float() / 255.0 - MNIST_MEAN) / MNIST_STD).view(B, 1, 28, 28)
    t = data.labels.cuda()
    for _ in range(n):
        tr.train_batch(x, t)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
