"""Time the fused step's kernels in isolation with HIP events (median of N launches)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.data.mnist import MNIST_MEAN, MNIST_STD  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402


def timeit(fn, n=200, reps=5):
    """Back-to-back launches (GPU never idles): per-launch average, median over reps."""
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / n)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    dev = torch.device("cuda")
    n = max(4096, B)
    eng = FusedLeNetTrainer(Net().to(dev), synthetic_mnist(n, seed=1), global_batch=B)
    eng.set_epoch_order(torch.randperm(n))
    ops = torch.ops.csed
    g = torch.empty(21840, device=dev)

    def train():
        ops.lenet_train(eng.train_data.images, eng.train_data.labels, eng.perm, eng.cursor, B, 0, eng.wimg,
                        eng.flat.data, eng.slab, eng.vslab, eng.loss_parts, 1.0 / B, MNIST_MEAN, MNIST_STD, 0.5, 1,
                        eng.rng_offset, eng.grid, eng.mfma, None, eng.xstage, eng.lstage, False)

    common = lambda: (eng.flat.data, eng.momentum_buf, eng.wimg, 0.01, 0.5, 0.0, 0.0, False, eng.step_count,
                      eng.ticket)

    def upd_full():
        ops.lenet_update(eng.slab, eng.grid, eng.vslab, B, None, None, *common(), None, None, True, eng.loss_parts,
                         eng.grid, eng.loss_acc, eng.mfma)

    def upd_reduce():
        ops.lenet_update(eng.slab, eng.grid, eng.vslab, B, None, g, *common(), None, None, False, None, 0, None,
                         eng.mfma)

    def upd_sgd_only():
        ops.lenet_update(eng.slab, eng.grid, eng.vslab, B, g, None, *common(), None, None, True, None, 0, None,
                         eng.mfma)

    zbuf = torch.empty(21840, device=dev)

    def pack():
        ops.lenet_pack(eng.flat.data, eng.wimg, eng.mfma)

    def empty():
        pass

    train()
    torch.cuda.synchronize()
    for name, fn in [("empty (event floor)", empty), ("lenet_train", train), ("update full", upd_full),
                     ("update reduce-only", upd_reduce), ("update sgd-only (grad_in)", upd_sgd_only),
                     ("pack images", pack), ("torch fill 21840", lambda: zbuf.zero_()),
                     ("train+update", lambda: (train(), upd_full()))]:
        print(f"B={B} {name:28s} {timeit(fn):8.2f} us")

    # s_memrealtime stamps (100 MHz) of one full update, relative to the
    # earliest block entry: shows dispatch skew and per-phase cost per role
    dbg = torch.zeros(8 * 256, dtype=torch.long, device=dev)
    for _ in range(3):
        train()
        dbg.zero_()
        ops.lenet_update(eng.slab, eng.grid, eng.vslab, B, None, None, *common(), None, None, True, eng.loss_parts,
                         eng.grid, eng.loss_acc, eng.mfma, dbg)
        torch.cuda.synchronize()
    st = dbg.view(256, 8).cpu().double()
    stamps(st, B, "after train")
    for _ in range(3):  # the update again, with nothing in between (its inputs unchanged)
        dbg.zero_()
        ops.lenet_update(eng.slab, eng.grid, eng.vslab, B, None, None, *common(), None, None, True, eng.loss_parts,
                         eng.grid, eng.loss_acc, eng.mfma, dbg)
        torch.cuda.synchronize()
    stamps(dbg.view(256, 8).cpu().double(), B, "after update")


def stamps(st, B, what):
    wpt = 1 if B <= 128 else (2 if B <= 256 else (4 if B <= 512 else 8))  # fc_waves_per_tile
    nfc = 88 if wpt == 1 else 88 // (8 // wpt)  # blocks [0, nfc) FC role, then 84 CONV role blocks
    nb = nfc + 84
    t0 = st[:nb, 0].min()
    rel = (st - t0) * 0.01  # us
    for role, sl, ks in [("CONV", slice(nfc, nb), [0, 1, 2, 3, 4]), ("FC", slice(0, nfc), [0, 1, 2, 3, 4])]:
        r = rel[sl]
        desc = "  ".join(f"s{k} med {r[:, k].median().item():.2f} max {r[:, k].max().item():.2f}" for k in ks)
        print(f"stamps {what} {role}: {desc}")
    # the slowest FC blocks (s4) and their tiles (lenet_fused.hip fc_tile_of_block: one tile
    # per block at this batch)
    if wpt == 1:
        def tile_of(b):
            q = 11 * (b % 8) + b // 8
            return (q % 4) * 21 + q // 4 if q < 84 else q
        fc = rel[:nfc, 4]
        order = sorted(range(nfc), key=lambda b: -fc[b].item())[:10]
        print(f"slowest FC blocks {what}: " + "  ".join(
            f"b{b}/t{tile_of(b)}(mt{tile_of(b) // 21 if tile_of(b) < 84 else 'fc2'},nt{tile_of(b) % 21 if tile_of(b) < 84 else tile_of(b) - 84})"
            f"={fc[b].item():.2f}/s1={rel[b, 1].item():.2f}" for b in order))


if __name__ == "__main__":
    main()
