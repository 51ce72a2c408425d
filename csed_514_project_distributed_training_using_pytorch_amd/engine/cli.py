"""Command-line trainers with the reference's contract.

* :func:`single_main` -- ``src/train.py``: 3 epochs, batch 64 / test 1000,
  SGD lr 0.01 momentum 0.5, log + checkpoint every 10 batches, test after
  every epoch, sample-image and loss-curve figures (ref src/train.py:10-117).
* :func:`dist_main` -- ``src/train_dist.py --local_rank R``: data-parallel,
  global batch 64 split over the ranks, DistributedSampler(seed=42)
  sharding, CrossEntropyLoss, lr 0.02, 6 epochs, per-epoch summary line,
  rank-0 ``model.pt`` (ref src/train_dist.py:58-164).

Defaults are the reference's; everything hard-coded there is a flag here
(world size / rank come from torchrun's environment or ``--local_rank``).
The GPU engine is ``fused`` (two HIP launches per step, HIP-graph replay) or
``modular`` (per-op HIP kernels + autograd + bucketed RCCL reducer); on a
CPU-only machine the same loops run on stock PyTorch ops.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch

from .. import ops
from ..data import DeviceLoader, get_mnist
from ..models import Net
from ..parallel.comm import all_reduce_max, barrier, destroy, init_distributed, replica_checksum
from ..parallel.sampler import ShardSampler
from ..utils import checkpoint, metrics, plot, prof


def _dtype(name: str) -> torch.dtype:
    return {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[name]


def _common_flags(ap: argparse.ArgumentParser) -> None:
    ap.add_argument("--data-root", default=None, help="MNIST root (default ./files/)")
    ap.add_argument("--synthetic", action="store_true", help="force synthetic data even if MNIST exists")
    ap.add_argument("--train-size", type=int, default=None, help="synthetic train set size (default 60000)")
    ap.add_argument("--test-size", type=int, default=None, help="synthetic test set size (default 10000)")
    ap.add_argument("--device", default=None, help="cuda | cpu (default: cuda if available)")
    ap.add_argument("--engine", choices=["fused", "modular"], default="fused")
    ap.add_argument("--dtype", choices=["bf16", "fp16", "fp32"], default="bf16",
                    help="GPU compute dtype: bf16 / fp16 MFMA operands with fp32 masters, or exact fp32 "
                         "(v_mfma_f32_16x16x4_f32, the reference's precision)")
    ap.add_argument("--no-plot", action="store_true")
    ap.add_argument("--out-dir", default=".", help="where images/, results/ and model.pt are written")


def _load_data(args, device):
    syn = True if args.synthetic else None
    train = get_mnist(args.data_root, train=True, synthetic=syn, n=args.train_size, seed=0)
    test = get_mnist(args.data_root, train=False, synthetic=syn, n=args.test_size, seed=0)
    return train, test


# ======================================================================== single
def single_main(argv=None) -> int:
    t0 = time.time()
    ap = argparse.ArgumentParser(description="single-process MNIST trainer (ref src/train.py)")
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--batch-size", type=int, default=64)
    ap.add_argument("--test-batch-size", type=int, default=1000)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--momentum", type=float, default=0.5)
    ap.add_argument("--log-interval", type=int, default=10)
    ap.add_argument("--ckpt-interval", type=int, default=None, help="batches between checkpoints "
                    "(default: every log line, as the reference)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--resume", action="store_true", help="load results/model.pth + optimizer.pth first")
    _common_flags(ap)
    args = ap.parse_args(argv)

    torch.backends.cudnn.enabled = False  # ref src/train.py:20 (our kernels never use MIOpen)
    torch.manual_seed(args.seed)
    ctx = init_distributed(world_size=1, device=args.device)
    dev = ctx.device
    out = args.out_dir
    ckpt_every = args.ckpt_interval or args.log_interval
    if dev.type == "cuda":
        ops.set_compute_dtype(_dtype(args.dtype))
    train, test_set = _load_data(args, dev)
    if train.synthetic:
        print("[csed] MNIST files not found: using synthetic 1x28x28 data of the same shape")
    test_loader = DeviceLoader(test_set, args.test_batch_size, shuffle=True, device=dev)
    if not args.no_plot:
        idx = torch.arange(min(6, len(test_set)))
        plot.plot_examples(test_set.images[idx].float().numpy(), test_set.labels[idx].numpy(),
                           os.path.join(out, "images/train_images.png"))

    net = Net().to(dev)
    hist = metrics.LossHistory()
    n_train = len(train)
    hist.test_counter = [i * n_train for i in range(args.epochs + 1)]
    use_fused = dev.type == "cuda" and args.engine == "fused"
    results = os.path.join(out, "results")

    if use_fused:
        from .fused import FusedLeNetTrainer

        eng = FusedLeNetTrainer(net, train, lr=args.lr, momentum=args.momentum, global_batch=args.batch_size,
                                compute_dtype=_dtype(args.dtype), seed=args.seed)
        opt_state = eng.optimizer_state_dict
        if args.resume:
            checkpoint.load_checkpoint(net, None, os.path.join(results, "model.pth"), None)
            eng.params_changed()
            eng.load_optimizer_state_dict(torch.load(os.path.join(results, "optimizer.pth"), weights_only=True))

        def test():
            lsum, correct = eng.evaluate(test_set)
            avg = lsum / len(test_set)
            hist.test_losses.append(avg)
            print(metrics.test_line(avg, correct, len(test_set), time.time() - t0))

        def save():
            checkpoint.save_model(net, os.path.join(results, "model.pth"))
            checkpoint._atomic_save(opt_state(), os.path.join(results, "optimizer.pth"))

        nb = (n_train + args.batch_size - 1) // args.batch_size
        test()
        for epoch in range(1, args.epochs + 1):
            order = torch.randperm(n_train)
            eng.set_epoch_order(order)
            full = eng.full_steps()

            def one_step(idx):
                if idx < full:
                    eng.run_steps(1)
                else:
                    eng.last_partial_step()

            done = 0
            while done < nb:
                logged = done % args.log_interval == 0
                ckpt = done % ckpt_every == 0
                if logged or ckpt:
                    # run this batch on its own so its loss is reported exactly (one host sync)
                    eng.take_loss()
                    one_step(done)
                    lsum, _ = eng.take_loss()
                    bsz = min(args.batch_size, n_train - done * args.batch_size)
                    if logged:
                        loss = lsum / bsz
                        print(metrics.train_line(epoch, done * bsz, n_train, 100.0 * done / nb, loss))
                        hist.train_losses.append(loss)
                        hist.train_counter.append(done * 64 + (epoch - 1) * n_train)
                    if ckpt:
                        save()
                    done += 1
                    continue
                # silent stretch up to the next logged/checkpointed batch: graph replays
                nxt = min(-(-done // args.log_interval) * args.log_interval, -(-done // ckpt_every) * ckpt_every, nb)
                k = min(nxt, full) - done
                if k > 0:
                    eng.run_steps(k)
                    done += k
                else:
                    one_step(done)
                    done += 1
            test()
    else:
        from .modular import ModularTrainer

        tr = ModularTrainer(net, lr=args.lr, momentum=args.momentum)
        if args.resume:
            checkpoint.load_checkpoint(net, tr.opt, os.path.join(results, "model.pth"),
                                       os.path.join(results, "optimizer.pth"))
        train_loader = DeviceLoader(train, args.batch_size, shuffle=True, device=dev,
                                    dtype=ops.compute_dtype() if dev.type == "cuda" else torch.float32)
        tr.bind_loader(train_loader)

        def test():
            total, correct, _ = tr.evaluate(test_loader)
            avg = total.item() / len(test_set)
            hist.test_losses.append(avg)
            print(metrics.test_line(avg, int(correct.item()), len(test_set), time.time() - t0))

        test()
        for epoch in range(1, args.epochs + 1):
            nb = len(train_loader)
            for batch_idx, (x, t) in enumerate(train_loader):
                loss = tr.train_batch(x, t, clone_loss=batch_idx % args.log_interval == 0)
                if batch_idx % args.log_interval == 0:
                    lv = loss.item()
                    print(metrics.train_line(epoch, batch_idx * len(x), n_train, 100.0 * batch_idx / nb, lv))
                    hist.train_losses.append(lv)
                    hist.train_counter.append(batch_idx * 64 + (epoch - 1) * n_train)
                if batch_idx % ckpt_every == 0:
                    checkpoint.save_checkpoint(net, tr.opt, os.path.join(results, "model.pth"),
                                               os.path.join(results, "optimizer.pth"))
            test()

    if not args.no_plot:
        plot.plot_loss_curve(hist.train_counter, hist.train_losses, hist.test_counter, hist.test_losses,
                             os.path.join(out, "images/train_test_curve.png"))
    return 0


# ========================================================================== dist
def _check_replicas(args, ctx, net, epoch: int) -> None:
    """--check-replicas E: every E epochs, all ranks must hold bitwise-identical parameters
    (the reference's DDP guarantees it; a divergence means a broken exchange)."""
    if not args.check_replicas or not ctx.is_distributed or (epoch + 1) % args.check_replicas:
        return
    flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()])
    ok, lo, hi = replica_checksum(ctx, flat)
    if not ok:
        raise SystemExit(f"replica check failed after epoch {epoch}: parameter hashes differ across ranks "
                         f"(min {lo}, max {hi})")
    if ctx.is_main:
        print(f"[csed] replica check after epoch {epoch}: parameters bitwise identical on {ctx.world_size} ranks "
              f"(hash {lo})", flush=True)


def dist_main(argv=None) -> int:
    t0 = time.time()  # ref: taken before rendezvous (src/train_dist.py:119)
    ap = argparse.ArgumentParser(description="data-parallel MNIST trainer (ref src/train_dist.py)")
    ap.add_argument("--local_rank", "--local-rank", type=int, default=None)
    ap.add_argument("--world-size", type=int, default=None)
    ap.add_argument("--epochs", type=int, default=6)
    ap.add_argument("--batch-size", type=int, default=64, help="GLOBAL batch (split over ranks)")
    ap.add_argument("--test-batch-size", type=int, default=1000)
    ap.add_argument("--lr", type=float, default=0.02)
    ap.add_argument("--momentum", type=float, default=0.5)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--sampler-seed", type=int, default=42)
    ap.add_argument("--backend", default=None, help="nccl (RCCL) | gloo (default: nccl on GPU)")
    ap.add_argument("--master-addr", default=None)
    ap.add_argument("--master-port", type=int, default=None)
    ap.add_argument("--bucket-mb", type=float, default=None,
                    help="gradient bucket cap of the modular engine's DDP reducer (default 25, one bucket); "
                         "rejected with --engine fused, whose exchange is fused into its update kernel")
    ap.add_argument("--check-replicas", type=int, default=0, metavar="E",
                    help="every E epochs, compare a bitwise hash of the parameters across ranks "
                         "(all-reduce MIN/MAX) and abort on divergence (0 = off)")
    ap.add_argument("--progress", action="store_true", help="tqdm bars (syncs every step, like the reference)")
    ap.add_argument("--inject-exchange-fault", type=int, default=None, metavar="EPOCH",
                    help="fault-injection test hook: in epoch EPOCH the last rank's exchange pushes go to a "
                         "dead-end buffer (its peers' waits time out); the epoch must be re-run on the "
                         "process-group all-reduce")
    ap.add_argument("--reference-metrics", action="store_true",
                    help="reproduce the reference's metric quirks (loss/bs sums, mean-of-batch-means val)")
    _common_flags(ap)
    args = ap.parse_args(argv)

    torch.backends.cudnn.enabled = False
    torch.manual_seed(args.seed)
    world = args.world_size or int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ["RANK"]) if "RANK" in os.environ else args.local_rank
    local = int(os.environ["LOCAL_RANK"]) if "LOCAL_RANK" in os.environ else args.local_rank
    ctx = init_distributed(rank=rank, world_size=world, local_rank=local, backend=args.backend,
                           master_addr=args.master_addr, master_port=args.master_port, device=args.device)
    dev = ctx.device
    if dev.type == "cuda":
        ops.set_compute_dtype(_dtype(args.dtype))
    if args.batch_size % ctx.world_size:
        raise SystemExit(f"global batch {args.batch_size} must be divisible by world size {ctx.world_size}")
    per_rank = args.batch_size // ctx.world_size
    use_fused = dev.type == "cuda" and args.engine == "fused"
    if use_fused and args.bucket_mb is not None:
        raise SystemExit("--bucket-mb applies to --engine modular only: the fused engine's gradient exchange "
                         "runs inside its update kernel (one 87 KB exchange per step, no buckets)")
    train, test_set = _load_data(args, dev)
    if train.synthetic and ctx.is_main:
        print("[csed] MNIST files not found: using synthetic 1x28x28 data of the same shape")
    sampler = ShardSampler(len(train), ctx.world_size, ctx.rank, shuffle=True, seed=args.sampler_seed)
    test_loader = DeviceLoader(test_set, args.test_batch_size, shuffle=True, device=dev)
    net = Net().to(dev)
    hist = metrics.LossHistory()
    # ref train_dist.py:89,153: counters in units of the whole training set (len(dataset))
    hist.test_counter = [i * len(train) for i in range(args.epochs)]
    bar = None
    if args.progress and ctx.is_main:
        try:
            from tqdm import tqdm as bar
        except ImportError:
            bar = None

    if use_fused:
        from .fused import FusedLeNetTrainer

        eng = FusedLeNetTrainer(net, train, lr=args.lr, momentum=args.momentum, global_batch=args.batch_size,
                                ctx=ctx, compute_dtype=_dtype(args.dtype), seed=args.seed)
        sampler.set_epoch(0)
        order = sampler.indices()
        i = 0
        while i < args.epochs:
            # the IPC exchange paths raise a device error word when a peer wait times out (the
            # kernel then finishes with an incomplete sum instead of hanging): snapshot the
            # training state so the epoch can be re-run on the process group's all-reduce
            ipc_live = ctx.is_distributed and eng.exch is not None
            snap = [t.clone() for t in eng._state()] if ipc_live else None
            if ipc_live and args.inject_exchange_fault == i and ctx.rank == ctx.world_size - 1:
                eng.inject_exchange_fault()
            n_hist = (len(hist.train_losses), len(hist.train_counter))
            eng.set_epoch_order(order)
            epoch_order = order
            steps, full, rem = eng.steps_per_epoch(), eng.full_steps(), eng.tail_size()
            with prof.range(f"train_epoch{i}"):
                if bar is not None:
                    it = bar(range(steps))
                    for s in it:
                        if s < full:
                            eng.run_steps(1)
                        else:
                            eng.last_partial_step()
                        lsum, _ = eng.take_loss()
                        bl = lsum / (per_rank if s < full else rem)  # ref: mean over data.shape[0]
                        it.set_description(f"training batch_loss={bl:.4f}")
                        hist.train_losses.append(bl)
                        hist.train_counter.append(s * 64 + i * len(train))
                    full_sum = sum(hist.train_losses[-steps:][:full]) * per_rank
                    tail_sum = hist.train_losses[-1] * rem if rem else 0.0
                else:
                    eng.run_steps(full)
                    if i + 1 < args.epochs:  # next epoch's order on the host while the graphs run
                        sampler.set_epoch(i + 1)
                        order = sampler.indices()
                    full_sum, _ = eng.take_loss()
                    eng.last_partial_step()
                    tail_sum, _ = eng.take_loss()
            if bar is not None and i + 1 < args.epochs:
                sampler.set_epoch(i + 1)
                order = sampler.indices()
            if ipc_live and int(all_reduce_max(ctx, float(eng.comm_errors()))):
                # some rank's peer wait timed out this epoch: its gradients are not the global
                # sum.  Every rank restores the epoch-start state, releases the IPC buffers
                # (collective) and re-runs the epoch on the process group's all-reduce (RCCL).
                if ctx.is_main:
                    print(f"[csed] epoch {i}: an IPC gradient exchange timed out waiting for a peer; "
                          "re-running the epoch on the process-group all-reduce", file=sys.stderr, flush=True)
                torch.cuda.synchronize(dev)
                for t, v in zip(eng._state(), snap):
                    t.copy_(v)
                eng.close()
                del hist.train_losses[n_hist[0]:], hist.train_counter[n_hist[1]:]
                order = epoch_order
                continue
            with prof.range(f"eval_epoch{i}"):
                vloss_sum, correct = eng.evaluate(test_set)
            n_test = len(test_set)
            if args.reference_metrics:
                # ref: sum over batches of (mean batch loss / batch size) (train_dist.py:86)
                train_loss = full_sum / per_rank / per_rank + (tail_sum / rem / rem if rem else 0.0)
                val_loss = vloss_sum / args.test_batch_size / n_test  # mean of batch means / dataset size
            else:
                train_loss = (full_sum + tail_sum) / len(sampler)
                val_loss = vloss_sum / n_test
            hist.test_losses.append(val_loss)
            acc = 100.0 * correct / n_test
            print(metrics.dist_epoch_line(i, train_loss, val_loss, acc, time.time() - t0), flush=True)
            _check_replicas(args, ctx, net, i)
            i += 1
        eng.close()
    else:
        from .modular import ModularTrainer

        tr = ModularTrainer(net, lr=args.lr, momentum=args.momentum, ctx=ctx, loss="ce",
                            bucket_cap_mb=25.0 if args.bucket_mb is None else args.bucket_mb)
        loader = DeviceLoader(train, per_rank, sampler=sampler, device=dev,
                              dtype=ops.compute_dtype() if dev.type == "cuda" else torch.float32)
        tr.bind_loader(loader)
        for i in range(args.epochs):
            sampler.set_epoch(i)
            losses = []
            it = loader if bar is None else bar(loader)
            for batch_idx, (x, t) in enumerate(it):
                loss = tr.train_batch(x, t)
                losses.append(loss)
                if bar is not None:
                    it.set_description(f"training batch_loss={loss.item():.4f}")
            ls = torch.stack(losses).double()
            hist.train_losses.extend(ls.tolist())
            hist.train_counter.extend(b * 64 + i * len(train) for b in range(len(losses)))
            total, correct, batch_means = tr.evaluate(test_loader)
            n_test = len(test_set)
            if args.reference_metrics:
                train_loss = (ls / per_rank).sum().item()
                val_loss = torch.stack(batch_means).sum().item() / n_test
            else:
                train_loss = ls.mean().item()
                val_loss = total.item() / n_test
            hist.test_losses.append(val_loss)
            acc = 100.0 * correct.item() / n_test
            print(metrics.dist_epoch_line(i, train_loss, val_loss, acc, time.time() - t0), flush=True)
            _check_replicas(args, ctx, net, i)

    barrier(ctx)
    if ctx.is_main:
        if not args.no_plot:
            plot.plot_loss_curve(hist.train_counter, hist.train_losses, hist.test_counter, hist.test_losses,
                                 os.path.join(args.out_dir, "images/train_test_curve_dist.png"))
        checkpoint.save_model(net, os.path.join(args.out_dir, "model.pt"))  # ref train_dist.py:163-164
    destroy()
    return 0
