"""Single-process MNIST training (ref src/train.py): 3 epochs, batch 64, SGD lr 0.01
momentum 0.5, log + checkpoint every 10 batches to results/, test after each epoch,
figures in images/.  Runs on one MI355X (fused HIP engine) or on the CPU.

    python src/train.py [--epochs 3] [--engine fused|modular] [--device cpu] [--synthetic] ...
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from csed_514_project_distributed_training_using_pytorch_amd.engine.cli import single_main  # noqa: E402

if __name__ == "__main__":
    sys.exit(single_main())
