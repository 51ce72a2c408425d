"""One-shot gradient all-reduce over HIP-IPC peer mappings (native: csrc/comm/).

Replaces, for the fused engine's single 87 KB gradient (ref
src/train_dist.py:83 -> DDP Reducer all-reduce), the ring/tree collective by a
kernel that reads every peer's buffer directly over its own xGMI link: one hop,
all 7 links of an MI355X at once, no host work, graph-capturable.

Bring-up is defensive.  Every rank creates its exchange buffer, the IPC handles
are all-gathered over the existing process group, each rank maps its peers and
runs a self-test: exact integer-valued sums over several rounds, the timeout
error word, and bitwise agreement with the process group's own all-reduce.  The
ranks then agree (MIN over the process group) and the path is enabled only if
every rank passed; otherwise callers keep using RCCL.  In ``auto`` mode the two
are then timed on the real buffer and the faster one is kept (the slowest
rank's numbers decide, so all ranks agree).  It is a standalone collective
(:func:`make_allreduce`, ``tools/allreduce_bench.py``, the loopback tests); the
fused engine does not train on it.

``CSED_ALLREDUCE`` selects the fused engine's gradient path: ``auto`` (default:
the in-kernel exchange if its self-test passes, else RCCL) | ``fused`` (the
in-kernel exchange or fail) | ``rccl`` (never try IPC).

The same IPC buffers also back the fused engine's in-kernel exchange
(:func:`open_exchange`): lenet_update pushes its reduced gradient to every peer
and sums all ranks itself, so a data-parallel step is one kernel fewer than
reduce + all-reduce + SGD.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from ..ops import _native
from .comm import DistContext, ctl_all_gather, ctl_all_gather_object, ctl_all_reduce, ctl_device


# latencies measured by the last auto selection (us per call, max over ranks), for reports
LAST_TIMING: dict | None = None
# why the last make_allreduce() fell back to the process group, for reports
LAST_NOTE: str | None = None


def _gather_handles(ctx: DistContext, h: torch.Tensor) -> torch.Tensor:
    mine = h.to(ctl_device(ctx))
    out = [torch.empty_like(mine) for _ in range(ctx.world_size)]
    ctl_all_gather(ctx, out, mine)
    return torch.stack([t.cpu() for t in out]).contiguous()


def _all_ok(ctx: DistContext, ok: bool) -> bool:
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=ctl_device(ctx))
    ctl_all_reduce(ctx, t, dist.ReduceOp.MIN)
    return bool(t.item())


class IpcAllReduce:
    """SUM all-reduce of one fp32 buffer of ``n`` elements across the process group.

    Construction is split so that every rank issues the same collectives even when
    a local step fails: :meth:`create` (local), :meth:`exchange` (collective:
    all-gather of the handles), :meth:`open` (local).  Use :func:`make_allreduce`.
    """

    def __init__(self, ctx: DistContext, n: int, blocks: int = 32, timeout_s: float | None = None):
        self.ctx = ctx
        self.n = int(n)
        self.n_pad = (self.n + 3) // 4 * 4
        self.blocks = int(blocks)
        self.timeout_s = float(timeout_s if timeout_s is not None else wait_timeout_s())
        self.id = -1
        self.measured_us: dict | None = None
        self.loopback_world = 0
        self._pad_in = self._pad_out = None
        if self.n_pad != self.n:
            self._pad_in = torch.zeros(self.n_pad, dtype=torch.float32, device=ctx.device)
            self._pad_out = torch.zeros_like(self._pad_in)

    def create(self) -> torch.Tensor:
        """Allocate the exchange buffer; returns this rank's IPC handle (CPU uint8)."""
        _native.require()
        with torch.cuda.device(self.ctx.device):
            self.id = int(torch.ops.csed.ipc_create(self.n_pad, self.blocks))
            return torch.ops.csed.ipc_handle(self.id)

    def exchange(self, handle: torch.Tensor) -> torch.Tensor:
        return _gather_handles(self.ctx, handle)

    def open(self, handles: torch.Tensor) -> None:
        with torch.cuda.device(self.ctx.device):
            torch.ops.csed.ipc_open(self.id, handles, self.ctx.rank)

    def open_loopback(self, world: int) -> None:
        """Map ``world`` virtual ranks onto this rank's own buffer (csrc/comm ipc_open_loopback):
        every exchange returns world x the local value, through the kernels' full push + poll
        code for world - 1 peers.  A one-GPU measurement of the world-N exchange's kernel side."""
        with torch.cuda.device(self.ctx.device):
            torch.ops.csed.ipc_open_loopback(self.id, int(world))
        self.loopback_world = int(world)

    def __call__(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """out = sum over ranks of x (in place when ``out`` is None).  Graph-capturable."""
        out = x if out is None else out
        ops = torch.ops.csed
        if self._pad_in is None:
            ops.ipc_allreduce(self.id, x, out, self.timeout_s)
        else:
            self._pad_in[: self.n].copy_(x)
            ops.ipc_allreduce(self.id, self._pad_in, self._pad_out, self.timeout_s)
            out.copy_(self._pad_out[: self.n])
        return out

    # error-word bits (csrc/comm/ipc_allreduce.h)
    ERR_TIMEOUT = 1
    ERR_MISMATCH = 2

    def error(self, reset: bool = False) -> int:
        """Error bits: ``ERR_TIMEOUT`` (a peer wait ran out), ``ERR_MISMATCH`` (loopback only:
        a received word carried the current tag but not the value its sender pushed)."""
        return int(torch.ops.csed.ipc_error(self.id, reset))

    def diag(self) -> dict | None:
        """The first loopback mismatch, as recorded in-kernel (None if there was none)."""
        d = list(torch.ops.csed.ipc_diag(self.id))
        if not d[0]:
            return None
        got = (d[5] & 0xFFFFFFFF) | ((d[6] & 0xFFFFFFFF) << 32)
        return {"block": d[1], "peer_row": d[2], "word": d[3], "tag": d[4] & 0xFFFFFFFF,
                "got_word": hex(got), "got_tag": d[6] & 0xFFFFFFFF, "want_bits": hex(d[7] & 0xFFFFFFFF),
                "poll_passes": d[8]}

    def mute(self, on: bool = True) -> None:
        """Fault injection: while on, this rank's pushes go to a dead-end buffer (csrc/comm
        ipc_set_mute), so its peers' waits time out as if it had died.  Launches resolved
        after the call see it (re-capture graphs)."""
        with torch.cuda.device(self.ctx.device):
            torch.ops.csed.ipc_set_mute(self.id, bool(on))

    def close(self) -> None:
        """Unmap the peers and free this rank's buffers (call after a process-group barrier,
        so that no peer is still pushing into them).  Idempotent."""
        if self.id >= 0:
            with torch.cuda.device(self.ctx.device):
                torch.ops.csed.ipc_destroy(self.id)
            self.id = -1

    def self_test(self, rounds: int = 4) -> bool:
        """Exact sums of integer-valued data over several rounds (both slot parities),
        no timeout, and bitwise agreement with the process group's all-reduce.

        Every rank must call it.  The process-group reductions run first, so a local
        failure in the IPC rounds cannot desynchronise the ranks' collectives; a rank
        that fails before its kernel makes its peers time out (error word), not hang.
        """
        ctx = self.ctx
        dev = ctx.device
        idx = torch.arange(self.n, device=dev, dtype=torch.float32)
        cases = []
        pg_dev = ctl_device(ctx)
        for r in range(rounds):
            x = torch.remainder(idx * (ctx.rank + 1) + r, 97.0)  # small integers: sums are exact in fp32
            z = x.to(pg_dev, copy=True)
            ctl_all_reduce(ctx, z)
            z = z.to(dev)
            exact = sum(torch.remainder(idx * (k + 1) + r, 97.0) for k in range(ctx.world_size))
            cases.append((x, z, exact))
        try:
            ok = True
            for x, z, exact in cases:
                y = self(x.clone())
                ok &= bool(torch.equal(y, exact)) and bool(torch.equal(y, z))
            torch.cuda.synchronize(dev)
            ok &= self.error(reset=True) == 0
        except Exception:
            ok = False
        return ok


# Ranks that may share one GPU and still run the spin-waiting exchange kernels.  Every rank's
# kernel must be resident at once (each waits for its peers' pushes): measured on one MI355X,
# 2 processes sharing the GPU run both paths (tests/test_comm_gpu.py), 4 did not (the
# self-test timed out: the GPU does not keep four processes' spinning kernels co-resident,
# profiles/dp_exchange_r1.md).  Beyond the limit the process group's all-reduce is used.
MAX_RANKS_PER_GPU = 2


def _device_key(ctx: DistContext) -> int:
    import hashlib
    import socket

    props = torch.cuda.get_device_properties(ctx.device)
    ident = getattr(props, "uuid", None)
    ident = str(ident) if ident is not None else f"{props.name}:{ctx.device.index}"
    digest = hashlib.sha1(f"{socket.gethostname()}|{ident}".encode()).digest()
    return int.from_bytes(digest[:7], "little")


def ranks_per_gpu(ctx: DistContext) -> int:
    """Largest number of ranks of the process group that drive the same physical GPU
    (collective).  One process per GPU gives 1."""
    mine = torch.tensor([_device_key(ctx)], dtype=torch.int64, device=ctl_device(ctx))
    keys = [torch.empty_like(mine) for _ in range(ctx.world_size)]
    ctl_all_gather(ctx, keys, mine)
    vals = [int(k.item()) for k in keys]
    return max(vals.count(v) for v in vals)


# Per-rank exchange diagnostics (bench.py JSON ``exchange_diag``, dpcheck's DPCHECK line): enough to
# name the failing stage of a data-parallel bring-up on a real node -- peer access of this rank's
# GPU, the IPC buffer's create / map, the exact self-test, the fused-vs-RCCL path timing, and at the
# end of a run the exchange's error word and first recorded mismatch.  Every rank reports every key
# (None where a stage did not run), so a report names the stage and the rank.
DIAG_KEYS = ("rank", "local_rank", "device", "device_count", "ranks_per_gpu", "peer_access", "ipc_open",
             "self_test", "path_timing_us", "allreduce", "note", "error_word", "first_mismatch")


def empty_diag(ctx: DistContext) -> dict:
    """This rank's diagnostics record with every stage unset."""
    d = dict.fromkeys(DIAG_KEYS)
    d.update(rank=ctx.rank, local_rank=int(os.environ.get("LOCAL_RANK", ctx.rank)),
             device=ctx.device.index if ctx.device.type == "cuda" else str(ctx.device))
    return d


def peer_access(device: torch.device) -> dict:
    """hipDeviceCanAccessPeer from ``device`` to every other visible GPU: {"i->j": bool}."""
    if device.type != "cuda":
        return {}
    i, n = device.index, torch.cuda.device_count()
    return {f"{i}->{j}": bool(torch.cuda.can_device_access_peer(i, j)) for j in range(n) if j != i}


def gather_diag(ctx: DistContext, local: dict) -> list[dict]:
    """Every rank's diagnostics, in rank order (collective; the local record alone at world 1)."""
    if not ctx.is_distributed:
        return [local]
    return ctl_all_gather_object(ctx, local)


def test_reject_hook() -> str:
    """``CSED_TEST_EXCH_REJECT`` (tests): ``open`` -- the last rank reports a failed buffer mapping;
    ``selftest`` -- its self-test fails.  The engine must fall back to the process group."""
    return os.environ.get("CSED_TEST_EXCH_REJECT", "").strip().lower()


def wait_timeout_s() -> float:
    """Wall-clock bound of every peer wait inside the exchange kernels (``CSED_IPC_TIMEOUT_S``,
    default 2 s): on expiry a kernel raises the comm error word and finishes instead of
    hanging the GPU."""
    return float(os.environ.get("CSED_IPC_TIMEOUT_S", "2.0"))


def allreduce_mode() -> str:
    """``CSED_ALLREDUCE``: auto (default) | fused | rccl (see engine/fused.py)."""
    mode = os.environ.get("CSED_ALLREDUCE", "auto").lower()
    if mode == "ipc":
        raise ValueError("CSED_ALLREDUCE=ipc was removed as a training path: the one-shot IPC kernel "
                         "depends on co-scheduling when ranks share a GPU and could not be tested "
                         "strictly; use auto / fused (the in-kernel exchange) or rccl")
    if mode not in ("auto", "fused", "rccl"):
        raise ValueError(f"CSED_ALLREDUCE={mode!r}: expected auto, fused or rccl")
    return mode


def _open(ctx: DistContext, n: int, blocks: int) -> tuple[IpcAllReduce | None, str]:
    """create -> vote -> all-gather handles -> open -> vote (every rank issues the same
    collectives whatever fails locally).  Returns the opened buffer, or None + why."""
    ar = IpcAllReduce(ctx, n, blocks=blocks)
    why = ""
    handle = None
    try:
        handle = ar.create()
    except Exception as e:
        why = f"create: {type(e).__name__}: {e}"
    ok = _all_ok(ctx, handle is not None)
    if ok:
        handles = ar.exchange(handle)
        try:
            ar.open(handles)
        except Exception as e:
            why, ok = f"open: {type(e).__name__}: {e}", False
        ok = _all_ok(ctx, ok)
    return (ar if ok else None), (why or ("" if ok else "a peer failed to create / map its buffer"))


def open_exchange(ctx: DistContext, words: int, shared: int | None = None) -> tuple[IpcAllReduce | None, str]:
    """An opened IPC exchange buffer of ``words`` 8-byte words per sender for a kernel that
    carries its own LL exchange (lenet_update's fused gradient all-reduce).  The caller
    self-tests it with that kernel.  Collective.  ``shared``: ranks_per_gpu(ctx) if known."""
    if not ctx.is_distributed or ctx.device.type != "cuda":
        return None, "not distributed on a GPU"
    shared = ranks_per_gpu(ctx) if shared is None else int(shared)
    if shared > MAX_RANKS_PER_GPU:
        return None, f"{shared} ranks share one GPU (spin-waiting exchange needs <= {MAX_RANKS_PER_GPU})"
    return _open(ctx, (words + 3) // 4 * 4, blocks=1)


def open_loopback_exchange(device: torch.device, words: int, world: int, blocks: int = 1) -> IpcAllReduce:
    """An exchange buffer of ``words`` 8-byte words per sender with ``world`` virtual ranks on
    ``device`` (see :meth:`IpcAllReduce.open_loopback`); ``blocks``: workgroups of its one-shot
    all-reduce kernel.  Local: no process group."""
    ar = IpcAllReduce(DistContext(device=device), (words + 3) // 4 * 4, blocks=blocks)
    ar.create()
    ar.open_loopback(world)
    return ar


def make_allreduce(ctx: DistContext, n: int, mode: str = "auto") -> IpcAllReduce | None:
    """The standalone one-shot IPC all-reduce if every rank can use it (see module docstring),
    else None.  ``mode``: ``auto`` (keep it only where it times faster than the process group)
    | ``ipc`` (use it; raise if unusable) | ``rccl`` (None).

    Every rank runs the same sequence of collectives whatever fails locally:
    create -> vote -> all-gather handles -> open -> vote -> self-test -> vote.
    """
    global LAST_NOTE
    if mode not in ("auto", "ipc", "rccl"):
        raise ValueError(f"make_allreduce mode {mode!r}: expected auto, ipc or rccl")
    if mode == "rccl" or not ctx.is_distributed or ctx.device.type != "cuda":
        return None
    shared = ranks_per_gpu(ctx)
    if shared > MAX_RANKS_PER_GPU:
        LAST_NOTE = f"ipc all-reduce off: {shared} ranks share one GPU (needs <= {MAX_RANKS_PER_GPU})"
        if mode == "ipc":
            raise RuntimeError(f"ipc all-reduce required but {LAST_NOTE}")
        return None
    if shared > 1 and mode != "ipc":
        # Ranks sharing a GPU (a rehearsal setup, never a real node): the auto mode keeps the
        # process group's all-reduce as the fallback.  Its spinning kernel depends on how the
        # GPU interleaves the processes' queues: tools/dp_step_bench.py --gloo still records one
        # 2 s timed-out wait per run on one shared MI355X (profiles/dp_exchange_r3.md), which the
        # fused exchange (one waiting point per step, inside lenet_update) does not show.
        LAST_NOTE = f"ipc all-reduce off: {shared} ranks share one GPU (auto mode; mode='ipc' forces it)"
        return None
    ar, why = _open(ctx, n, blocks=32)
    ok = ar is not None
    if ok:
        ok = _all_ok(ctx, ar.self_test())
        why = why or ("" if ok else "self-test mismatch or timeout on some rank")
    if not ok:
        if mode == "ipc":
            raise RuntimeError(f"ipc all-reduce required but it is unusable ({why or 'a peer failed'})")
        LAST_NOTE = f"ipc all-reduce off: {why or 'a peer failed'}"
        return None
    if mode == "auto" and ctx.backend == "nccl":
        # keep whichever is faster on this machine (slowest rank decides, all ranks agree)
        global LAST_TIMING
        t_ipc, t_pg = _time_both(ctx, ar)
        ar.measured_us = LAST_TIMING = {"ipc_us": round(t_ipc, 2), "rccl_us": round(t_pg, 2)}
        if t_pg < t_ipc:
            return None
    return ar


def _time_both(ctx: DistContext, ar: IpcAllReduce, calls: int = 50) -> tuple[float, float]:
    """Per-call latency (us, max over ranks) of the IPC kernel and of the process group's
    all-reduce on the same 87 KB buffer, eager launches back to back."""
    dev = ctx.device
    x = torch.randn(ar.n, device=dev)

    def run(fn) -> float:
        for _ in range(5):
            fn()
        torch.cuda.synchronize(dev)
        dist.barrier(device_ids=[dev.index])
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(calls):
            fn()
        b.record()
        b.synchronize()
        t = torch.tensor([a.elapsed_time(b) * 1e3 / calls], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    t_ipc = run(lambda: ar(x))
    t_pg = run(lambda: dist.all_reduce(x))
    return t_ipc, t_pg
