"""Wall-clock timelines (s_memrealtime, 100 MHz) of the one-kernel step (csed::lenet_step)
and of the two-kernel step (lenet_train + lenet_update), relative to the first training
workgroup's start: training workgroups' start / end, update workgroups' start / end of
wait (one-kernel) / loads done / finish.  Also times back-to-back eager launches.
usage: python tools/step_timeline.py [B]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.data.mnist import MNIST_MEAN, MNIST_STD  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402


def med(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    dev = torch.device("cuda")
    eng = FusedLeNetTrainer(Net().to(dev), synthetic_mnist(B * 400, seed=1), global_batch=B)
    eng.set_epoch_order(torch.randperm(B * 400))
    ops = torch.ops.csed
    dbg = torch.zeros(B * 32, dtype=torch.long, device=dev)
    udbg = torch.zeros(8 * 256, dtype=torch.long, device=dev)

    def one(d=None, u=None):
        ops.lenet_step(eng.train_data.images, eng.train_data.labels, eng.perm, eng.cursor, B, 0, eng.wimg,
                       eng.flat.data, eng.slab, eng.vslab, eng.loss_parts, 1.0 / B, MNIST_MEAN, MNIST_STD, 0.5, 1,
                       eng.rng_offset, eng.mfma, eng.xstage, eng.lstage, eng.momentum_buf, 0.01, 0.5, 0.0, 0.0,
                       False, eng.step_count, eng.ticket, eng.loss_acc, eng.bar, d, u)

    def two(d=None, u=None):
        ops.lenet_train(eng.train_data.images, eng.train_data.labels, eng.perm, eng.cursor, B, 0, eng.wimg,
                        eng.flat.data, eng.slab, eng.vslab, eng.loss_parts, 1.0 / B, MNIST_MEAN, MNIST_STD, 0.5, 1,
                        eng.rng_offset, B, eng.mfma, d, eng.xstage, eng.lstage, True)
        ops.lenet_update(eng.slab, B, eng.vslab, B, None, None, eng.flat.data, eng.momentum_buf, eng.wimg, 0.01,
                         0.5, 0.0, 0.0, False, eng.step_count, eng.ticket, eng.cursor, eng.rng_offset, True,
                         eng.loss_parts, B, eng.loss_acc, eng.mfma, u)

    for name, fn in (("one kernel", one), ("two kernels", two)):
        rows = {}
        for it in range(60):
            udbg.zero_()
            fn(dbg, udbg)
            torch.cuda.synchronize()
            if it < 10:
                continue
            st = dbg.view(B, 32).cpu().tolist()
            ud = udbg.view(256, 8).cpu().tolist()
            up = [r for r in ud if r[0] != 0 and r[4] != 0 or (r[0] != 0 and r[3] != 0)]
            t0 = min(r[22] for r in st)
            vals = {"train WG start": [r[22] - t0 for r in st], "train WG end": [r[23] - t0 for r in st],
                    "update WG start": [r[0] - t0 for r in up],
                    "update WG loads done": [r[1] - t0 for r in up],
                    "update WG finish": [max(r[3], r[4]) - t0 for r in up]}
            if name == "one kernel":
                nfc = int(os.environ.get("CSED_FC_TPB_COUNT", "88"))  # FC workgroups come first
                for role, rr in (("FC", up[:nfc]), ("CONV", up[nfc:])):
                    for si, nm in ((5, "go"), (1, "loads"), (2, "s2"), (3, "s3"), (4, "s4")):
                        vals[f"{role} {nm}"] = [r[si] - t0 for r in rr]
                nupd = len(up)
                tr = ud[nupd:nupd + B]
                vals["train WG signal"] = [r[1] - t0 for r in tr]
                vals["train WG counted"] = [r[2] - t0 for r in tr]
                vals["update WG go seen"] = [r[5] - t0 for r in up]
            for k, v in vals.items():
                rows.setdefault(k, ([], []))
                rows[k][0].append(med(v))
                rows[k][1].append(max(v))
        print(f"B={B} {name}: us from the first training WG's start (median over 50 launches)")
        for k, (m, l) in rows.items():
            print(f"  {k:22s} median-WG {med(m) / 100:6.2f}   last-WG {med(l) / 100:6.2f}")
    assert eng.bar[2].item() == 0

    def timeit(fn, n=400, reps=5):
        ts = []
        for _ in range(reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(n):
                fn()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) * 1e3 / n)
        return med(ts)

    print(f"back-to-back eager launches: one kernel {timeit(one):.2f} us, two kernels {timeit(two):.2f} us")


if __name__ == "__main__":
    main()
