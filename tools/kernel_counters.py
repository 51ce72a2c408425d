"""Launch the fused step's two kernels N times each (no graph), for rocprofv3 --pmc runs.

    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU ... --output-format csv -d OUT -o run -- \
        python3 tools/kernel_counters.py [B] [N]

then `python tools/kernel_counters.py --summarize OUT/run_counter_collection.csv` prints the
per-dispatch mean of every counter for lenet_train / lenet_update.
"""
import csv
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(B: int, n: int):
    import torch

    from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist
    from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer
    from csed_514_project_distributed_training_using_pytorch_amd.models import Net

    dev = torch.device("cuda")
    torch.manual_seed(1)
    eng = FusedLeNetTrainer(Net().to(dev), synthetic_mnist(4096, seed=1), global_batch=B)
    eng.set_epoch_order(torch.randperm(4096))
    for _ in range(n):
        eng.step()
    torch.cuda.synchronize()


def short_name(name: str) -> str:
    """A kernel's function name without namespaces / template arguments / parameters."""
    import re

    if name.startswith("_Z"):  # mangled: _ZN <len><id> ... (the last id is the function) or _Z <len><id>
        i = 3 if name.startswith("_ZN") else 2
        last = None
        while i < len(name) and name[i].isdigit():
            j = i
            while j < len(name) and name[j].isdigit():
                j += 1
            n = int(name[i:j])
            last, i = name[j:j + n], j + n
        return last or name[:40]
    base = re.sub(r"<.*", "", name.replace("(anonymous namespace)", "").split("(")[0])
    return base.split("::")[-1].replace("void ", "").strip() or name[:40]


def summarize(path: str):
    """Per-dispatch mean of every counter per kernel (the fused step's kernels by role, every other
    kernel -- e.g. the modular engine's -- by its short name; the runtime's copy / fill kernels out)."""
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name", "")
        short = ("lenet_train" if "lenet_train" in name else "lenet_tile" if "lenet_tile" in name
                 else "lenet_update" if "lenet_update" in name else short_name(name))
        if "rocclr" in name or "at::native" in name:
            continue
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(f"== {k}")
        for c, v in sorted(cs.items()):
            print(f"  {c:28s} {sum(v) / len(v):14.1f}   (n={len(v)})")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--summarize":
        for p in sys.argv[2:]:
            summarize(p)
    else:
        run(int(sys.argv[1]) if len(sys.argv) > 1 else 64, int(sys.argv[2]) if len(sys.argv) > 2 else 200)
