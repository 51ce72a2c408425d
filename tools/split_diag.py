"""Split-step stage-6/7 timeline (diagnostic stamps WSTAMP in lenet_fused.hip, split builds only):
cycles from the stage-6 start of each workgroup, median over workgroups."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda")
data = synthetic_mnist(4096, seed=1)
torch.manual_seed(1)
eng = FusedLeNetTrainer(Net().to(dev), data, global_batch=B)
eng.set_epoch_order(torch.randperm(4096))
dbg = torch.zeros(eng.grid * 32, dtype=torch.long, device=dev)
for _ in range(20):
    eng.gradient(eng.grid, dbg)
torch.cuda.synchronize()
st = dbg.view(eng.grid, 32).cpu().double()
names = {9: "wave0 past wgrad/stores", 26: "wave12 wgrad MFMAs done", 27: "wave12 at barrier6", 24: "wave0 dgrad MFMAs done",
         25: "wave0 SCR written", 28: "wave4 SCR written", 29: "wave11 SCR written", 7: "stage7 start",
         30: "wave0 combine done", 31: "wave12 stores done", 8: "stage8 start", 14: "sample end"}
for k, nm in names.items():
    print(f"{nm:28s} {(st[:, k] - st[:, 6]).median().item():8.0f}")
