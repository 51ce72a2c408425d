"""Kernel-side cost of lenet_update's fused gradient exchange at world N = 1 / 2 / 4 / 8 on ONE
GPU (loopback mode: the N - 1 virtual peers are sender slots of this rank's own receive buffer,
csrc/comm ipc_open_loopback), at the per-rank batches of the reference's strong-scaling
config (global batch 64 over N ranks, ref src/train_dist.py:133) and at 64.

    python tools/exchange_loopback.py [B ...]

Per (B, N): the update kernel alone (back-to-back launches, HIP events), a whole training step
(graph replays of train + update), and s_memrealtime stamps of the update's blocks (us from the
earliest block entry: s3 = gradient final in its lane, s4 = exchanged + SGD done).  What the
loopback does not contain is the xGMI flight time of the pushes (one one-way hop).

The timing runs the update kernel a real world-N step runs: the loopback invariant check (which
has its own kernel instantiations, +0.4 / +0.7 us at N = 4 / 8, profiles/round5.md) is switched
off here (CSED_LOOPBACK_CHECK=0) unless the caller sets the variable; the exchange tests run
with it on."""
import os
import sys

os.environ.setdefault("CSED_LOOPBACK_CHECK", "0")  # (read by csrc/comm at the first exchange)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402


def timeit(fn, n=200, reps=5):
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


def step_us(eng, nsteps=32, reps=10):
    g = eng._capture(nsteps)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / (reps * nsteps)


def main():
    batches = [int(b) for b in sys.argv[1:]] or [8, 16, 32, 64]
    dev = torch.device("cuda")
    data = synthetic_mnist(8192, seed=1)
    ops = torch.ops.csed
    rows = []
    for B in batches:
        for N in (1, 2, 4, 8):
            torch.manual_seed(1)
            eng = FusedLeNetTrainer(Net().to(dev), data, lr=0.02, momentum=0.5, global_batch=B,
                                    loopback_world=N if N > 1 else 0)
            eng.set_epoch_order(torch.randperm(len(data)))
            eng.step()
            torch.cuda.synchronize()
            common = (eng.flat.data, eng.momentum_buf, eng.wimg, eng.lr, eng.momentum, eng.dampening,
                      eng.weight_decay, eng.nesterov, eng.step_count, eng.ticket)
            xid = eng.exch.id if eng.exch is not None else -1

            def upd(dbg=None):
                ops.lenet_update(eng.slab, eng.grid, eng.vslab, B, None, None, *common, None, None, True,
                                 eng.loss_parts, eng.grid, eng.loss_acc, eng.mfma, dbg, xid, eng.exch_timeout_s)

            t_upd = timeit(upd)
            t_step = step_us(eng)
            dbg = torch.zeros(8 * 256, dtype=torch.long, device=dev)
            meds = {}
            for _ in range(3):
                eng.step()  # fresh slabs, then the stamped update
                dbg.zero_()
                upd(dbg)
                torch.cuda.synchronize()
            st = dbg.view(256, 8).double()
            live = st[:, 0] > 0
            st = st[live]
            rel = (st - st[:, 0].min()) * 0.01
            for k in (3, 4):
                meds[k] = (rel[:, k].median().item(), rel[:, k].max().item())
            err = eng.comm_errors()
            rows.append((B, N, t_upd, t_step, meds[3], meds[4], err))
            print(f"B={B:3d} N={N} update {t_upd:6.2f} us  step {t_step:6.2f} us  "
                  f"stamps s3 med {meds[3][0]:.2f} max {meds[3][1]:.2f}  s4 med {meds[4][0]:.2f} "
                  f"max {meds[4][1]:.2f}  comm_errors {err}", flush=True)
            eng.close()
            del eng
    print("\n| per-rank B | N | update kernel us | step us (graph) | exchange cost vs N=1, update / step | "
          "s3 max | s4 max |")
    print("|---:|---:|---:|---:|---:|---:|---:|")
    base = {(b, 1): (u, s) for b, n, u, s, *_ in rows if n == 1}
    for B, N, u, s, m3, m4, err in rows:
        bu, bs = base[(B, 1)]
        print(f"| {B} | {N} | {u:.2f} | {s:.2f} | {u - bu:+.2f} / {s - bs:+.2f} | {m3[1]:.2f} | {m4[1]:.2f} |")


if __name__ == "__main__":
    main()
