"""Per-stage cycle shares of the fused LeNet train kernel (diagnostic build path).

Runs lenet_train with the `dbg` stamp buffer: thread 0 of every workgroup
records s_memtime at kernel start, after the per-WG preamble and at the start
of each stage of its first sample.  Prints median cycles per stage over WGs.
Stamps serialise a little; read the shares, not the absolute total.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402

NAMES = ["start->first stage", "pixels+masks+prefetch", "conv1", "conv2", "fc1", "fc2+loss+dZ1",
         "dP2 (MFMA-tr)+pool2 bwd", "conv2 wgrad", "conv2 dgrad", "dgrad tile-8 reduce", "conv1 wgrad"]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    grid = int(sys.argv[2]) if len(sys.argv) > 2 else B
    dev = torch.device("cuda")
    data = synthetic_mnist(4096, seed=1)
    torch.manual_seed(1)
    eng = FusedLeNetTrainer(Net().to(dev), data, global_batch=B, grid=grid)
    eng.set_epoch_order(torch.randperm(4096))
    dbg = torch.zeros(grid * 16, dtype=torch.long, device=dev)
    for _ in range(20):
        eng.gradient(grid, dbg)
    torch.cuda.synchronize()
    st = dbg.view(grid, 16).cpu().double()
    # order: 12 = kernel start, 0..8 = stage starts (9 = dgrad inside stage 6), 11 = after all samples
    seq = [12, 0, 1, 2, 3, 4, 5, 6, 9, 7, 8, 11]
    d = torch.stack([st[:, seq[i + 1]] - st[:, seq[i]] for i in range(len(seq) - 1)], 1)
    med = d.median(0).values
    tot = (st[:, 11] - st[:, 12]).median().item()
    print(f"B={B} grid={grid}: median total {tot:.0f} cycles (s_memtime ticks)")
    # preamble stamps: 12 kernel start (wave 0), 10 LDS-DMA issued (wave 0), 15 small
    # loads issued (wave 4), 13 = 14 preamble end (wave 0), 0 first stage (after the barrier)
    pre = [(st[:, 10] - st[:, 12]).median().item(), (st[:, 15] - st[:, 12]).median().item(),
           (st[:, 13] - st[:, 12]).median().item(), (st[:, 0] - st[:, 14]).median().item()]
    print(f"  preamble (from kernel start): DMA issued {pre[0]:.0f}, small loads issued {pre[1]:.0f}, "
          f"wave 0 done {pre[2]:.0f}; then to stage0 (barrier) {pre[3]:.0f}")
    for n, v in zip(NAMES, med.tolist()):
        print(f"  {n:24s} {v:8.0f}  {100 * v / tot:5.1f}%")


if __name__ == "__main__":
    main()
