"""Process-group bootstrap and point-to-point helpers.

Ref: ``init_process_group("gloo", rank, world_size)`` with a hard-coded
``MASTER_ADDR=10.128.0.2`` (src/train_dist.py:144-146) and the 2-machine
send/recv smoke test (src/run1.py:8-24).

Here one process drives one MI355X.  The backend is RCCL (PyTorch's "nccl"
backend on ROCm) whenever the process owns a GPU, so collectives run over
xGMI; gloo remains for CPU-only runs and tests.  Rendezvous follows the
torchrun environment contract (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR,
MASTER_PORT) with the reference's ``--local_rank`` convention accepted too,
and 127.0.0.1 as the default master address.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str | None = None
    # control plane: a gloo group over every rank for the bring-up's and the bench's small host
    # collectives (votes, handle / diagnostics gathers, the initial parameter broadcast, timing
    # maxima, barriers) when the RCCL communicator is created lazily (init_distributed(lazy_rccl=
    # True)): RCCL's communicator takes 1.0 s (warm) to 3.6 s (fresh box) to create, even for one
    # rank (tools/rccl_init_probe.py, profiles/r6/rehearsal), and a data-parallel step whose
    # gradients travel over the in-kernel IPC exchange never needs it -- it is created at its first
    # collective: the fallback all-reduce or the fused-vs-RCCL path timing
    control: object = None

    @property
    def is_distributed(self) -> bool:
        return self.backend is not None and self.world_size > 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def env_int(name: str, default: int | None) -> int | None:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def _gpu_count() -> int:
    # device_count() does not initialise the HIP runtime on this image
    try:
        return torch.cuda.device_count()
    except Exception:
        return 0


def _wait_listening(addr: str, port: int, timeout_s: float) -> None:
    import socket
    import time

    t_end = time.time() + timeout_s
    while True:
        try:
            with socket.create_connection((addr, port), timeout=1.0):
                return
        except OSError:
            if time.time() > t_end:
                return  # (the rendezvous below reports the failure with torch's own error)
            time.sleep(0.001)


def rendezvous(world_size: int | None = None, rank: int | None = None, timeout_s: float = 600.0):
    """The job's TCPStore (torch's env:// rendezvous: MASTER_ADDR / MASTER_PORT, torchrun's agent
    store when it runs under torchrun) and a barrier on it: returns once every rank has connected.
    Touches no GPU, so a rank can wait here for the others (their imports finish at different
    times) while its HIP context comes up in another thread; ``init_distributed(store=...)`` then
    builds the process group on it.  None at world size 1."""
    world_size = world_size if world_size is not None else env_int("WORLD_SIZE", 1)
    if world_size <= 1:
        return None
    if rank is None:
        rank = env_int("RANK", None)
        rank = rank if rank is not None else (env_int("LOCAL_RANK", 0) or 0)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    if rank != 0 and os.environ.get("TORCHELASTIC_USE_AGENT_STORE") != "True":
        # rank 0 hosts the store (no torchrun agent store): wait until it listens, polling every
        # millisecond -- a TCPStore client that finds no server backs off for up to a second per
        # retry, which a rank whose imports finished first paid in full (0.65 s of rendezvous
        # measured with 2 CPU ranks, profiles/r6/rehearsal)
        _wait_listening(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), timeout_s)
    store, _, _ = next(dist.rendezvous("env://", rank, world_size, timeout=datetime.timedelta(seconds=timeout_s)))
    if store.add("csed/rdzv/arrived", 1) == world_size:
        store.set("csed/rdzv/all", "1")
    store.wait(["csed/rdzv/all"])
    return store


def init_distributed(rank: int | None = None, world_size: int | None = None, local_rank: int | None = None,
                     backend: str | None = None, master_addr: str | None = None, master_port: int | None = None,
                     device: str | None = None, timeout_s: float = 600.0, store=None,
                     lazy_rccl: bool = False, set_device: bool = True) -> DistContext:
    """Initialise the default process group (if world_size > 1) and pick this rank's device.
    ``store``: a store from :func:`rendezvous` (the process group is built on it: no second
    rendezvous).  ``lazy_rccl`` (RCCL backend): no eager communicator -- it is created at the
    first RCCL collective -- and a gloo group over every rank becomes the context's control
    plane (``DistContext.control``).  ``set_device=False``: leave torch.cuda.set_device to the
    caller (a lazy-RCCL process group touches no GPU, so it can come up while another thread
    creates the HIP context)."""
    world_size = world_size if world_size is not None else env_int("WORLD_SIZE", 1)
    rank = rank if rank is not None else env_int("RANK", None)
    local_rank = local_rank if local_rank is not None else env_int("LOCAL_RANK", None)
    if rank is None:
        rank = local_rank if local_rank is not None else 0
    if local_rank is None:
        local_rank = rank
    ngpu = _gpu_count()
    if device is None:
        device = "cuda" if ngpu > 0 else "cpu"
    if device.startswith("cuda"):
        if ngpu == 0:
            raise RuntimeError("device=cuda requested but no GPU is visible")
        dev = torch.device("cuda", local_rank % ngpu)
        if set_device:
            torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    be = None
    if world_size > 1:
        be = backend or ("nccl" if dev.type == "cuda" else "gloo")
        os.environ.setdefault("MASTER_ADDR", master_addr or "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(master_port or 29500))
        if master_addr:
            os.environ["MASTER_ADDR"] = master_addr
        if master_port:
            os.environ["MASTER_PORT"] = str(master_port)
        control = None
        if not dist.is_initialized():
            kw = {}
            if be == "nccl" and not lazy_rccl:
                kw["device_id"] = dev
            if store is not None:
                kw["store"] = store
            dist.init_process_group(be, rank=rank, world_size=world_size,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
            if be == "nccl" and lazy_rccl:
                control = dist.new_group(backend="gloo")  # (collective: every rank, same order)
        return DistContext(rank, world_size, local_rank, dev, be, control)
    return DistContext(rank, world_size, local_rank, dev, be)


def ctl_device(ctx: DistContext) -> torch.device:
    """Device of the control plane's tensors: the host when a gloo group carries them."""
    if ctx.control is not None or ctx.backend != "nccl":
        return torch.device("cpu")
    return ctx.device


def ctl_all_reduce(ctx: DistContext, t: torch.Tensor, op=None) -> torch.Tensor:
    """All-reduce of a control-plane tensor (on ``ctl_device``) over every rank, in place."""
    dist.all_reduce(t, op=op if op is not None else dist.ReduceOp.SUM, group=ctx.control)
    return t


def ctl_all_gather(ctx: DistContext, out: list, t: torch.Tensor) -> list:
    dist.all_gather(out, t, group=ctx.control)
    return out


def ctl_all_gather_object(ctx: DistContext, obj) -> list:
    out: list = [None] * ctx.world_size
    dist.all_gather_object(out, obj, group=ctx.control)
    return out


def ctl_broadcast(ctx: DistContext, t: torch.Tensor, src: int = 0) -> torch.Tensor:
    """Broadcast of a device tensor from ``src`` over the control plane (through the host when
    that is gloo)."""
    if ctl_device(ctx).type == t.device.type:
        dist.broadcast(t, src=src, group=ctx.control)
        return t
    host = t.cpu()
    dist.broadcast(host, src=src, group=ctx.control)
    t.copy_(host)
    return t


def destroy() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()


def quiesce() -> None:
    """Block until every process group's watchdog has retired its outstanding collectives.

    Call right before a HIP graph capture.  The watchdog thread polls each pending collective's
    completion event; HIP refuses an event query while the event's stream is capturing
    (``hipErrorCapturedEvent``), and the watchdog then aborts the process -- a race with the
    watchdog's ~100 ms poll that a capture shortly after a collective (the warm-up step's
    all-reduces, the initial parameter broadcast) could lose.  Collectives issued inside a capture
    are not handed to the watchdog, so an empty list stays empty for the capture.
    """
    if not (dist.is_available() and dist.is_initialized()):
        return
    try:
        groups = list(dist.distributed_c10d._world.pg_map.keys())
    except AttributeError:  # (private registry moved: the default group at least)
        groups = [dist.group.WORLD]
    for pg in groups:
        try:
            pg._wait_for_pending_works()
        except (AttributeError, RuntimeError, NotImplementedError):  # (gloo / older builds: nothing to wait for)
            pass


def barrier(ctx: DistContext) -> None:
    if ctx.is_distributed:
        if ctx.control is not None:
            dist.barrier(group=ctx.control)
        elif ctx.backend == "nccl":
            dist.barrier(device_ids=[ctx.device.index])
        else:
            dist.barrier()


def p2p_exchange(ctx: DistContext, src: int = 0, dst: int = 1) -> torch.Tensor:
    """The reference smoke test (src/run1.py:8-17): rank ``src`` adds 1 to a zeros(1)
    tensor and sends it; rank ``dst`` receives it.  Returns the local tensor."""
    t = torch.zeros(1, device=ctx.device)
    if ctx.rank == src:
        t += 1
        dist.send(t, dst=dst)
    elif ctx.rank == dst:
        dist.recv(t, src=src)
    return t


def all_reduce_max(ctx: DistContext, value: float) -> float:
    """Max of a host scalar over ranks (used to report the slowest rank's time)."""
    if not ctx.is_distributed:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=ctl_device(ctx))
    ctl_all_reduce(ctx, t, dist.ReduceOp.MAX)
    return float(t.item())


def replica_checksum(ctx: DistContext, t: torch.Tensor) -> tuple[bool, int, int]:
    """Bitwise replica check: a position-weighted int64 hash of ``t``'s bit
    pattern, reduced with MIN and MAX over the ranks.  Equal on every rank iff (up to hash
    collisions) every replica holds the same bytes.  Returns (equal, min, max); collective."""
    flat = t.detach().reshape(-1)
    bits = flat.view(torch.int32) if flat.dtype == torch.float32 else flat.float().view(torch.int32)
    w = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) * 2 + 1
    h = (bits.to(torch.int64) * w).sum()  # int64 arithmetic wraps: deterministic
    if not ctx.is_distributed:
        v = int(h.item())
        return True, v, v
    dev = ctl_device(ctx)
    lo, hi = h.to(dev).clone(), h.to(dev).clone()
    ctl_all_reduce(ctx, lo, dist.ReduceOp.MIN)
    ctl_all_reduce(ctx, hi, dist.ReduceOp.MAX)
    return bool(lo.item() == hi.item()), int(lo.item()), int(hi.item())
