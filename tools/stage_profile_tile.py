"""Per-stage cycles of the sample-tile train kernel (csrc/kernels/lenet_tile.hip), diagnostic
stamps of the first tile of every workgroup (s_memtime; median over workgroups).

    python tools/stage_profile_tile.py [B ...]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402

NAMES = ["preamble", "(loop entry)", "0 pixels+masks", "1 conv1", "2 conv2", "3 fc1", "4 loss",
         "5 dP2+pool2 bwd", "6 conv2 wgrad+dgrad", "7 conv1 wgrad"]


def main():
    for B in [int(b) for b in sys.argv[1:]] or [1024, 8192]:
        dev = torch.device("cuda")
        n = max(4096, B)
        torch.manual_seed(1)
        eng = FusedLeNetTrainer(Net().to(dev), synthetic_mnist(n, seed=1), global_batch=B,
                                compute_dtype=torch.float16)
        eng.set_epoch_order(torch.randperm(n))
        grid = eng.grid
        dbg = torch.zeros(grid * 32, dtype=torch.long, device=dev)
        for _ in range(10):
            eng.gradient(grid, dbg)
        torch.cuda.synchronize()
        st = dbg.view(grid, 32).cpu().double()
        seq = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10]
        d = [st[:, 1] - st[:, 0]] + [st[:, seq[i + 1]] - st[:, seq[i]] for i in range(1, len(seq) - 1)]
        d = torch.stack(d, 1).median(0).values.tolist()
        tot = (st[:, 11] - st[:, 0]).median().item()
        tile = (st[:, 10] - st[:, 2]).median().item()
        print(f"tile kernel B={B} grid={grid}: kernel {tot:.0f} cycles, first tile {tile:.0f} (median over WGs)")
        for name, v in zip(NAMES, d):
            print(f"  {name:22s} {v:8.0f}")
        px = (st[:, 14] - st[:, 2]).median().item()
        print(f"  (stage 0: staged pixels in and written after {px:.0f} cycles)")
        arr = [(st[:, 16 + w] - st[:, 2]).median().item() for w in range(16)]
        print("  stage-0 barrier arrival per wave (cycles after stage start): " + " ".join(f"{v:.0f}" for v in arr))
        # workgroup start / end skew on the 100 MHz realtime clock (10 ns ticks, all XCDs)
        t0, t1 = st[:, 12], st[:, 13]
        base = t0.min()
        start, end, dur = (t0 - base) * 0.01, (t1 - base) * 0.01, (t1 - t0) * 0.01
        q = torch.tensor([0.0, 0.5, 0.9, 1.0], dtype=torch.double)
        print(f"  realtime (us): span {end.max().item():.2f}; start p0/50/90/100 "
              f"{' / '.join(f'{v:.2f}' for v in start.quantile(q).tolist())}; per-WG duration p0/50/90/100 "
              f"{' / '.join(f'{v:.2f}' for v in dur.quantile(q).tolist())}; end p0/50/90/100 "
              f"{' / '.join(f'{v:.2f}' for v in end.quantile(q).tolist())}")


if __name__ == "__main__":
    main()
