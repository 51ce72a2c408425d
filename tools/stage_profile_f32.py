"""Per-stage cycles of the exact-fp32 train kernel (csrc/kernels/lenet_fused_f32.hip), diagnostic
stamps: thread 0 of every workgroup records s_memtime at kernel entry, after the preamble, at each
stage start of its first sample, at that sample's end and at the kernel's end.  Median over
workgroups; read the shares (the stamps serialise a little).

    python tools/stage_profile_f32.py [B ...]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402

NAMES = ["preamble", "(sample loop entry)", "0 pixels+masks", "1 conv1", "2 conv2", "3 fc1 (VALU)",
         "4 fc2+loss+dZ1", "5 dP2 (VALU)+pool2 bwd", "6 conv2 wgrad+dgrad", "7 dgrad combine",
         "8 conv1 wgrad (VALU)"]


def main():
    for B in [int(b) for b in sys.argv[1:]] or [64, 8]:
        dev = torch.device("cuda")
        n = max(4096, 2 * B)
        torch.manual_seed(1)
        eng = FusedLeNetTrainer(Net().to(dev), synthetic_mnist(n, seed=1), global_batch=B,
                                compute_dtype=torch.float32)
        eng.set_epoch_order(torch.randperm(n))
        grid = eng.grid
        dbg = torch.zeros(grid * 32, dtype=torch.long, device=dev)
        for _ in range(20):
            eng.gradient(grid, dbg)
        torch.cuda.synchronize()
        st = dbg.view(grid, 32).cpu().double()
        seq = list(range(0, 12))
        d = torch.stack([st[:, seq[i + 1]] - st[:, seq[i]] for i in range(len(seq) - 1)], 1)
        med = d.median(0).values.tolist()
        tot = (st[:, 12] - st[:, 0]).median().item()
        print(f"fp32 B={B} grid={grid}: kernel {tot:.0f} cycles (median over workgroups)")
        for name, v in zip(NAMES, med):
            print(f"  {name:26s} {v:8.0f}  {100 * v / tot:5.1f}%")
        if grid == 4 * B:  # split step: workgroup g is part g // B of sample g % B
            parts = [d[p * B:(p + 1) * B].median(0).values.tolist() for p in range(4)]
            print("  per part (median):   " + "  ".join(f"{'part ' + str(p):>8s}" for p in range(4)))
            for i, name in enumerate(NAMES):
                print(f"  {name:22s} " + "  ".join(f"{parts[p][i]:8.0f}" for p in range(4)))
        # workgroup start / end skew on the 100 MHz realtime clock (10 ns ticks, all XCDs)
        t0, t1 = st[:, 13], st[:, 14]
        base = t0.min()
        start, end, dur = (t0 - base) * 0.01, (t1 - base) * 0.01, (t1 - t0) * 0.01
        q = torch.tensor([0.0, 0.5, 0.9, 1.0], dtype=torch.double)
        print(f"  realtime (us): span {end.max().item():.2f}; start p0/50/90/100 "
              f"{' / '.join(f'{v:.2f}' for v in start.quantile(q).tolist())}; per-WG duration p0/50/90/100 "
              f"{' / '.join(f'{v:.2f}' for v in dur.quantile(q).tolist())}")


if __name__ == "__main__":
    main()
