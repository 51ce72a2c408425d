"""`Net` -- the reference model (ref src/model.py:4-22), re-exported from the
MI355X-native package so `from model import Net` keeps working in these scripts.
Parameter names/shapes/init are identical; the GPU forward runs fused HIP kernels."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from csed_514_project_distributed_training_using_pytorch_amd.models.net import Net  # noqa: E402,F401
