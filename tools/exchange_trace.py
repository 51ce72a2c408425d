"""Where the loopback exchange's step time goes: a graph of stamped steps (train + update with
their s_memrealtime stamps on, 100 MHz wall clock shared by every kernel) at per-rank batch B
and virtual world N (csrc/comm ipc_open_loopback), and the same graph without stamps for the
step time.

    python tools/exchange_trace.py [--batch 8] [--worlds 1 2 8] [--steps 32]

Per step (medians over the graph's steps, us): train = first train workgroup entry -> last
train workgroup exit; gap_tu = last train exit -> first update block entry; upd_s3 / upd_s4 =
first update entry -> last block's gradient final (s3) / exchanged + SGD done (s4); gap_ut =
last update s4 -> next step's first train entry.  The update kernel's own end (its stores
drained, the dispatch retired) falls inside gap_ut.

At per-rank batches that take the sample-tile kernel (csrc/kernels/lenet_tile.hip, B >=
tile_min_batch()) "train" is lenet_tile's span (its realtime stamps 12 / 13) and the update grid
is fc_blocks(B) + 84 blocks (the FC blocks first): e.g. --batch 1024 8192 --worlds 1."""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.data.mnist import MNIST_MEAN, MNIST_STD  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import (  # noqa: E402
    FusedLeNetTrainer, tile_grid, tile_min_batch)
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402


def stamped_graph(eng, nsteps, dt, du):
    ops = torch.ops.csed
    B, grid = eng.B, eng.grid
    kern = eng.kernel_for(B, grid)
    st = eng._stages(kern)
    common = (eng.flat.data, eng.momentum_buf, eng.wimg, eng.lr, eng.momentum, eng.dampening,
              eng.weight_decay, eng.nesterov, eng.step_count, eng.ticket)
    xid = eng.exch.id if eng.exch is not None else -1

    def step(i):
        ops.lenet_train(eng.train_data.images, eng.train_data.labels, eng.perm, eng.cursor, B, 0, eng.wimg,
                        eng.flat.data, eng.slab, eng.vslab, eng.loss_parts, eng._train_scale(eng.grad_scale),
                        MNIST_MEAN, MNIST_STD, eng.drop_p, eng.seed, eng.rng_offset, grid, eng.mfma, dt[i],
                        eng.xstage if st else None, eng.lstage if st else None, st, kern)
        ops.lenet_update(eng.slab, grid, eng.vslab, B, None, None, *common, eng.cursor, eng.rng_offset, True,
                         eng.loss_parts, grid, eng.loss_acc, eng.mfma, du[i], xid, eng.exch_timeout_s,
                         eng._post_scale(eng.grad_scale), eng.fc_part)

    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step(0)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        for i in range(nsteps):
            step(i)
    torch.cuda.synchronize()
    return g


def graph_step_us(eng, nsteps, reps=10):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[8])
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 8])
    ap.add_argument("--steps", type=int, default=32)
    args = ap.parse_args()
    dev = torch.device("cuda")
    data = synthetic_mnist(max(8192, 4 * max(args.batch)), seed=1)
    print("| B | N | step us (graph) | train | gap train->upd | upd s3 | upd s4 | FC s4 | CONV s4 | "
          "gap upd s4->next train | sum | FC push->done | FC passes | CONV push->done | CONV passes |")
    print("|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for B in args.batch:
        for N in args.worlds:
            torch.manual_seed(1)
            eng = FusedLeNetTrainer(Net().to(dev), data, lr=0.02, momentum=0.5, global_batch=B,
                                    loopback_world=N if N > 1 else 0)
            eng.set_epoch_order(torch.randperm(len(data)))
            eng.step()
            torch.cuda.synchronize()
            t_step = graph_step_us(eng, args.steps)
            n = args.steps
            dt = torch.zeros(n, eng.grid * 32, dtype=torch.long, device=dev)
            du = torch.zeros(n, 8 * 1024, dtype=torch.long, device=dev)
            kern = eng.kernel_for(B, eng.grid)
            tile = B >= tile_min_batch() and kern != 1 and eng.grid == tile_grid(B)
            i_in, i_out = (12, 13) if tile else (22, 23)
            # fc_blocks(B) (lenet_fused.hip): 88 FC tiles, 8 / waves-per-tile of them per block
            wpt = 1 if B <= 128 else 2 if B <= 256 else 4 if B <= 512 else 8
            nfc = 88 if (N > 1 or wpt == 1) else 88 // (8 // wpt)
            # split-K fc gradients (B > 1024, no exchange): 88 x S FC blocks, S = B / 1024 as a
            # power of two <= 8 (lenet_fused.hip fc_split_slices; CSED_FC_SLICES forces it)
            if N == 1 and B > 1024 and eng.fc_part is not None:
                forced = int(os.environ.get("CSED_FC_SLICES", "0") or 0)
                S = 1
                while S * 2 <= 8 and (S * 2 <= forced if forced > 0 else S * 2 * 1024 <= B):
                    S *= 2
                nfc = 88 * S
            g = stamped_graph(eng, n, dt, du)
            for _ in range(3):
                dt.zero_()
                du.zero_()
                g.replay()
                torch.cuda.synchronize()
            T = dt.view(n, eng.grid, 32).double().cpu()
            U = du.view(n, 1024, 8).double().cpu()
            rows, xrows = [], []
            for i in range(n - 1):
                t0, t1 = T[i, :, i_in].min().item(), T[i, :, i_out].max().item()
                u = U[i]
                u0 = u[:, 0][u[:, 0] > 0].min().item()
                s3 = u[:, 3].max().item()
                s4 = u[:, 4][u[:, 4] > 0].max().item()
                # blocks [0, nfc): the FC role, then the 84 CONV blocks
                fc_r, cv_r = slice(0, nfc), slice(nfc, nfc + 84)
                fc4 = u[fc_r, 4][u[fc_r, 4] > 0].max().item()
                cv4 = u[cv_r, 4][u[cv_r, 4] > 0].max().item()
                nt0 = T[i + 1, :, i_in].min().item()
                rows.append(((t1 - t0) * 0.01, (u0 - t1) * 0.01, (s3 - u0) * 0.01, (s4 - u0) * 0.01,
                             (fc4 - u0) * 0.01, (cv4 - u0) * 0.01, (nt0 - s4) * 0.01, (nt0 - t0) * 0.01))
                # exchange stamps (ll_allreduce): 5 = pushes issued, 6 = poll passes; per role, the
                # median block's push -> exchange done and its mean pass count
                x = []
                for rr in (fc_r, cv_r):
                    r = u[rr]
                    ok = r[:, 5] > 0
                    if ok.any():
                        x += [statistics.median(((r[ok, 4] - r[ok, 5]) * 0.01).tolist()), r[ok, 6].mean().item()]
                    else:
                        x += [float("nan"), float("nan")]
                xrows.append(x)
            med = [statistics.median(c) for c in zip(*rows)]
            xmed = [statistics.median(c) for c in zip(*xrows)]
            print(f"| {B} | {N} | {t_step:.2f} | " + " | ".join(f"{m:.2f}" for m in med) + " | " +
                  " | ".join("-" if m != m else f"{m:.2f}" for m in xmed) + " |", flush=True)
            if os.environ.get("TRACE_DUMP"):
                torch.save({"T": T, "U": U}, f"{os.environ['TRACE_DUMP']}_B{B}_N{N}.pt")
            print(f"  comm_errors {eng.comm_errors()}", flush=True)
            eng.close()
            del eng, g


if __name__ == "__main__":
    main()
