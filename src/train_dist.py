"""Data-parallel MNIST training (ref src/train_dist.py): one process per MI355X, RCCL
gradient all-reduce over xGMI, DistributedSampler(seed=42) sharding, global batch 64,
SGD lr 0.02 momentum 0.5, 6 epochs, per-epoch summary line, rank 0 writes model.pt.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 src/train_dist.py
    python src/train_dist.py --local_rank R --world-size N      (reference-style, env MASTER_ADDR)
    python -m csed_514_project_distributed_training_using_pytorch_amd.parallel.launch --nproc 8 src/train_dist.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from csed_514_project_distributed_training_using_pytorch_amd.engine.cli import dist_main  # noqa: E402

if __name__ == "__main__":
    sys.exit(dist_main())
