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

NAMES = ["preamble end->stage 0", "pixels+masks+prefetch", "conv1", "conv2", "fc1", "fc2+loss+dZ1",
         "dP2 (MFMA-tr)+pool2 bwd", "conv2 wgrad", "conv2 dgrad", "dgrad tile-8 reduce", "conv1 wgrad"]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    grid = int(sys.argv[2]) if len(sys.argv) > 2 else None  # default: the engine's (split step: 4 * B)
    dev = torch.device("cuda")
    n = max(4096, 2 * B)
    data = synthetic_mnist(n, seed=1)
    torch.manual_seed(1)
    eng = FusedLeNetTrainer(Net().to(dev), data, global_batch=B, grid=grid)
    grid = eng.grid
    eng.set_epoch_order(torch.randperm(n))
    dbg = torch.zeros(grid * 48, dtype=torch.long, device=dev)  # 32 stamp slots + 16 wave entries
    for _ in range(20):
        eng.gradient(grid, dbg)
    torch.cuda.synchronize()
    st = dbg[:grid * 32].view(grid, 32).cpu().double()
    ent = dbg[grid * 32:].view(grid, 16).cpu().double()
    # Stamps (thread 0): 12 kernel start, 10 LDS-DMA issued, 17 / 16 wave 4 start / small loads consumed,
    # 13 preamble end, 0..8 stage starts of the stamped sample (9 = dgrad inside stage 6),
    # 14 end of the stamped sample, 11 after all samples.  The stamped sample is sample 1
    # when a workgroup has several (steady state), else sample 0.
    seq = [13, 0, 1, 2, 3, 4, 5, 6, 9, 7, 8, 14]
    d = torch.stack([st[:, seq[i + 1]] - st[:, seq[i]] for i in range(len(seq) - 1)], 1)
    med = d.median(0).values
    tot = (st[:, 11] - st[:, 12]).median().item()
    per = (st[:, 14] - st[:, 0]).median().item()
    print(f"B={B} grid={grid}: median kernel {tot:.0f} cycles (s_memtime ticks), stamped sample {per:.0f}")
    pre = [(st[:, 10] - st[:, 12]).median().item(), (st[:, 13] - st[:, 12]).median().item()]
    ld = [(st[:, 17] - st[:, 12]).median().item(), (st[:, 16] - st[:, 12]).median().item()]
    print(f"  preamble (from kernel start): DMA issued {pre[0]:.0f}, wave 4 starts {ld[0]:.0f}, small loads "
          f"consumed {ld[1]:.0f}; wave 0 done {pre[1]:.0f}")
    bar = [(st[:, k] - st[:, 12]).median().item() for k in (15, 21, 1, 2)]
    print(f"  wave 4 at the preamble barrier {bar[0]:.0f}; weight DMA landed (wave 0, end of conv1) {bar[1]:.0f}; "
          f"conv1 start {bar[2]:.0f}, conv2 start {bar[3]:.0f}")
    dma = [(st[:, 17 + w] - st[:, 12]).median().item() for w in (1, 2, 3)]
    arr = [(st[:, 24 + w] - st[:, 12]).median().item() for w in range(8)]
    print(f"  DMA issued by waves 1-3: {dma}; waves 0-7 reach the first barrier: {arr}")
    if ent.abs().sum() > 0:  # every wave's first instruction (s_memtime), relative to the earliest wave
        e0 = ent.min(1, keepdim=True).values
        rel = (ent - e0).median(0).values.tolist()
        print("  wave entry (cycles after the workgroup's first wave): " + " ".join(f"{v:.0f}" for v in rel))
        print(f"  kernel-start stamp (12) after the first wave's entry: {(st[:, 12] - e0[:, 0]).median().item():.0f}")
    span = (st[:, 14] - st[:, 13]).median().item()
    for name, v in zip(NAMES, med.tolist()):
        print(f"  {name:24s} {v:8.0f}  {100 * v / span:5.1f}%")


if __name__ == "__main__":
    main()
