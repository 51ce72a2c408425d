"""Realtime phase stamps of lenet_update per workgroup (USTAMP in csrc/kernels/lenet_fused.hip:
a.dbg[blk * 8 + k] = s_memrealtime, 100 MHz, one clock for every XCD), for the FC and CONV roles.

    python tools/update_stamps.py [B ...]

Stamp k per role -- FC: 0 entry, 1 K loop done (chunk path) / first tile, 2 after the tile
combine, 3 SGD applied, 4 exchange / stores done; CONV: 0 entry, 1 slab loads issued, 2 reduced,
3 combined, 4 SGD + images written.  Times in us from the earliest entry of the launch.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402


def main():
    ops = torch.ops.csed
    for B in [int(b) for b in sys.argv[1:]] or [64, 1024]:
        dev = torch.device("cuda")
        n = max(4096, 2 * B)
        torch.manual_seed(1)
        dt = torch.float16 if B >= 1024 else torch.bfloat16
        eng = FusedLeNetTrainer(Net().to(dev), synthetic_mnist(n, seed=1), global_batch=B, compute_dtype=dt)
        eng.set_epoch_order(torch.randperm(n))
        nblk = ops.lenet_layout()[-1] if False else 256
        dbg = torch.zeros(nblk * 8, dtype=torch.long, device=dev)
        g = torch.empty(21840, device=dev)
        for _ in range(10):
            eng.gradient()
            ops.lenet_update(eng.slab, eng.grid, eng.vslab, B, None, g, eng.flat.data, eng.momentum_buf, eng.wimg,
                             eng.lr, eng.momentum, eng.dampening, eng.weight_decay, eng.nesterov, eng.step_count,
                             eng.ticket, None, None, False, eng.loss_parts, eng.grid, eng.loss_acc, eng.mfma, dbg)
        torch.cuda.synchronize()
        st = dbg.view(nblk, 8).cpu().double()
        live = st[:, 0] > 0
        st = st[live]
        base = st[:, 0].min()
        t = (st - base) * 0.01
        t[st == 0] = float("nan")
        nfc = int(os.environ.get("NFC", "88"))
        for name, rows in (("FC", t[:nfc]), ("CONV", t[nfc:])):
            if len(rows) == 0:
                continue
            med = [rows[:, k][~rows[:, k].isnan()].median().item() if (~rows[:, k].isnan()).any() else float("nan")
                   for k in range(5)]
            mx = [rows[:, k][~rows[:, k].isnan()].max().item() if (~rows[:, k].isnan()).any() else float("nan")
                  for k in range(5)]
            print(f"B={B} {name:4s} blocks {len(rows):3d}  stamp median " + " ".join(f"{v:6.2f}" for v in med)
                  + "   max " + " ".join(f"{v:6.2f}" for v in mx))


if __name__ == "__main__":
    main()
