"""N eager full-batch steps of the fused engine (for kernel traces): python tools/step_loop.py [B] [N]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
N = int(sys.argv[2]) if len(sys.argv) > 2 else 300
eng = FusedLeNetTrainer(Net().cuda(), synthetic_mnist(B * (N + 1), seed=1), global_batch=B)
eng.set_epoch_order(torch.randperm(B * (N + 1)))
eng.run_steps(N, use_graph=False)
torch.cuda.synchronize()
print(eng.step_kind, eng.step_count.item())
