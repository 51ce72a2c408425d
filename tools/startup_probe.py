"""Where bench.py's time_elapsed_s goes: wall clock of each startup phase (import, GPU
context, synthetic data, engine + graph capture, epoch 0)."""
import time

T0 = time.time()
import os  # noqa: E402
import sys  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

t_import = time.time()
torch.zeros(1, device="cuda")
torch.cuda.synchronize()
t_ctx = time.time()
from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402

t_pkg = time.time()
train = synthetic_mnist(60000, seed=0)
test = synthetic_mnist(10000, seed=0, train=False)
t_data = time.time()
torch.manual_seed(1)
eng = FusedLeNetTrainer(Net().cuda(), train, lr=0.02, momentum=0.5, global_batch=64)
eng.set_epoch_order(torch.randperm(60000))
t_eng = time.time()
eng.prepare(32, ks=(eng.full_steps(), 20))
torch.cuda.synchronize()
t_cap = time.time()
eng.run_steps(eng.full_steps(), 32)
eng.last_partial_step()
eng.evaluate(test)
torch.cuda.synchronize()
t_ep = time.time()
print(f"import torch {t_import - T0:.3f}  gpu context {t_ctx - t_import:.3f}  package {t_pkg - t_ctx:.3f}  "
      f"data {t_data - t_pkg:.3f}  engine {t_eng - t_data:.3f}  capture {t_cap - t_eng:.3f}  "
      f"epoch0 {t_ep - t_cap:.3f}  total {t_ep - T0:.3f} s (threads {torch.get_num_threads()})")
