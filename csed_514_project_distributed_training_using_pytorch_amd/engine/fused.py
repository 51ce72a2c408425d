"""Fused LeNet training engine: the MI355X fast path for ``Net`` (ref src/model.py).

One training step = two HIP kernels (``csed::lenet_train`` + ``csed::lenet_update``,
see csrc/kernels/lenet_fused.hip) at any world size:

    lenet_train    per-sample fwd+bwd of the whole network in LDS -> per-WG gradient slabs
    lenet_update   fixed-order slab reduce -> [world > 1: in-kernel exchange with every
                   peer over xGMI, rank-ordered sum] -> SGD-momentum + fp32 master params
                   + 16-bit weight images + device counters

The data-parallel gradient all-reduce (ref src/train_dist.py:83, DDP's one
87,360-byte bucket) is fused into lenet_update: each update lane pushes its
rank-local gradient value straight into every peer's IPC-mapped receive buffer
and sums what the peers pushed (csrc/comm buffers, LL-tagged words).  It is
enabled after a collective bring-up and an exact self-test; if either fails, or
``CSED_ALLREDUCE=rccl`` asks for it, the step runs as the fallback

    lenet_update (reduce only) -> RCCL all-reduce -> SGD kernel

In ``auto`` mode with one rank per GPU (a real node, pushes over xGMI) both
steps are then timed at bring-up -- one 16-step graph each -- and the faster is
kept, so a fused exchange slower than RCCL is never locked in (SURVEY §7.3 step
6).  ``CSED_TIME_PATHS``: ``auto`` (default: time exactly then), ``1`` (always
time, also on ranks sharing a GPU, and also time an exchange-free step), ``0``
(never: a passing self-test keeps the fused path).

All per-step state (batch cursor into this rank's epoch permutation, Philox
offset, optimizer step) lives on the device, so a sequence of steps is
captured once into a HIP graph and replayed with no host work per step.

The model's parameters are re-homed into the engine's flat fp32 buffer, so the
``Net`` module always sees the current weights (checkpointing, evaluation
through the op library, ``state_dict()``) without copies.
"""
from __future__ import annotations

import math
import os
import sys

import torch
import torch.distributed as dist

from ..data.mnist import MNIST_MEAN, MNIST_STD, MNISTData
from ..models.net import N_PARAMS, Net
from ..ops import _native
from ..parallel import comm as _comm
from ..parallel.comm import DistContext
from ..parallel import ipc as _ipc
from ..parallel.ipc import allreduce_mode, open_exchange, open_loopback_exchange, wait_timeout_s
from ..utils.flat import FlatParams

N_VEC = 464  # per-sample fc vector length (kernels/lenet_layout.h VEC)


_HIP_LIBS: list | None = None


def _hip_libs() -> list:
    """ctypes handles of the HIP runtime this process already loaded (via torch), never a second
    copy."""
    global _HIP_LIBS
    if _HIP_LIBS is None:
        import ctypes

        try:
            with open("/proc/self/maps") as f:
                paths = {ln.split()[-1] for ln in f if "libamdhip64.so" in ln}
            _HIP_LIBS = [ctypes.CDLL(p) for p in sorted(paths)]
        except OSError:
            _HIP_LIBS = []
    return _HIP_LIBS


def _clear_hip_error() -> None:
    """Reset this thread's sticky HIP error after a failed stream capture.  Our ops report
    ``hipGetLastError()`` after each launch, so an invalidated capture would otherwise
    surface as a failure of the next (eager) launch."""
    for lib in _hip_libs():
        lib.hipGetLastError()


class NativeGraph:
    """A step graph captured with ``torch.classes.csed.HipGraph`` (csrc/bindings.cpp), replayed by
    one ctypes ``hipGraphLaunch`` on the current stream (the ScriptObject keeps the graph alive)."""

    _launch = None

    def __init__(self, obj, device: torch.device):
        import ctypes

        self.obj = obj
        self.device_index = device.index
        self.exec = ctypes.c_void_p(obj.exec_handle())
        if NativeGraph._launch is None:
            fn = _hip_libs()[0].hipGraphLaunch
            fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int
            NativeGraph._launch = fn

    def replay(self) -> None:
        e = NativeGraph._launch(self.exec, torch._C._cuda_getCurrentRawStream(self.device_index))
        if e != 0:
            raise RuntimeError(f"hipGraphLaunch failed ({e})")

    def num_nodes(self) -> int:
        return int(self.obj.num_nodes())


def _hip_graph_upload(exec_handle: int, stream: int) -> bool:
    """hipGraphUpload of an instantiated graph on a stream (CSED_GRAPH_UPLOAD=1)."""
    import ctypes

    fn = _hip_libs()[0].hipGraphUpload
    fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int
    return fn(ctypes.c_void_p(exec_handle), ctypes.c_void_p(stream)) == 0


def layout() -> tuple[int, int, int, int]:
    """Buffer sizes of the fused kernels, from the extension (csrc/kernels/lenet_fused.hip):
    16-bit weight-image elements (I_END), conv slab row per workgroup (CNP_PAD: conv1.w/b +
    conv2.w/b = 5280 floats in 64-float chunks), per-sample fc vector length (VEC) and the
    largest per-rank batch that uses batch staging (STAGE_MAXB)."""
    wimg, conv, vec, nparams, stage_max, *_ = (int(v) for v in torch.ops.csed.lenet_layout())
    assert nparams == N_PARAMS
    return wimg, conv, vec, stage_max


def split_factor() -> int:
    """Workgroups per sample of the split step (csed::lenet_train KS)."""
    return int(torch.ops.csed.lenet_layout()[6])


def tile_samples() -> int:
    """Samples per tile of the sample-tile training kernel (csrc/kernels/lenet_tile.hip)."""
    _native.require()
    return int(torch.ops.csed.lenet_layout()[7])


def tile_min_batch() -> int:
    """Smallest per-rank batch the auto mode runs on the sample-tile kernel."""
    _native.require()
    return int(torch.ops.csed.lenet_layout()[8])


def tile_grid(B: int) -> int:
    """Workgroups of the sample-tile kernel at per-rank batch B."""
    return min(256, -(-B // tile_samples()))


def exch_words() -> int:
    """8-byte words per sender of lenet_update's fused exchange buffer."""
    return int(torch.ops.csed.lenet_layout()[5])


def native_max_steps() -> int:
    """Longest run of full steps launched by the native executor instead of a graph replay
    (``CSED_NATIVE_STEPS``; 0 = always graphs).  See ``FusedLeNetTrainer.step_plan``."""
    return int(os.environ.get("CSED_NATIVE_STEPS", "0"))


class FusedLeNetTrainer:
    def __init__(self, model: Net, train: MNISTData, lr: float = 0.01, momentum: float = 0.5,
                 dampening: float = 0.0, weight_decay: float = 0.0, nesterov: bool = False,
                 global_batch: int = 64, ctx: DistContext | None = None,
                 compute_dtype: torch.dtype = torch.bfloat16, drop_p: float = 0.5, seed: int = 1,
                 grid: int | None = None, broadcast_init: bool = True, comm: bool | None = None,
                 split: bool | None = None, loopback_world: int = 0,
                 reuse_exchange: "FusedLeNetTrainer | None" = None):
        import time

        _native.require()
        t_init = time.perf_counter()
        self.bringup_s: dict[str, float] = {}  # bring-up phases (s), for the bench JSON
        self.ctx = ctx or DistContext(device=next(model.parameters()).device)
        self.device = self.ctx.device
        if self.device.type != "cuda":
            raise RuntimeError("FusedLeNetTrainer runs on a GPU")
        self.model = model
        self.world = self.ctx.world_size if self.ctx.is_distributed else 1
        # comm=True forces the all-reduce path even at world size 1 (tests RCCL graph capture
        # on a single GPU); default: collectives exactly when there is more than one rank
        self.comm = (self.world > 1) if comm is None else (bool(comm) and dist.is_initialized())
        if global_batch % self.world:
            raise ValueError(f"global batch {global_batch} not divisible by world size {self.world}")
        self.global_batch = int(global_batch)
        self.B = self.global_batch // self.world
        self.grid = int(grid) if grid else min(self.B, 256)
        if compute_dtype not in _native.MFMA_CODE:
            raise ValueError(f"compute dtype {compute_dtype}: expected bfloat16, float16 or float32")
        self.lr, self.momentum, self.dampening = float(lr), float(momentum), float(dampening)
        self.weight_decay, self.nesterov = float(weight_decay), bool(nesterov)
        self.mfma = _native.MFMA_CODE[compute_dtype]
        self.compute_dtype = compute_dtype
        self.drop_p = float(drop_p)
        self.seed = int(seed)  # masks decorrelate across ranks through the rank id in the element index
        self.train_data = train.to(self.device)
        dev = self.device
        self.bringup_s["data_to_device"] = time.perf_counter() - t_init

        self.flat = FlatParams(list(model.parameters()))
        if self.flat.numel != N_PARAMS:
            raise ValueError("FusedLeNetTrainer needs the reference Net architecture")
        if broadcast_init and self.world > 1:  # the DDP-constructor parameter sync (CS4)
            _comm.ctl_broadcast(self.ctx, self.flat.data, src=0)  # (RCCL, or the host over gloo)
        self.momentum_buf = _native.zeros(self.flat.data.shape, torch.float32, self.flat.data.device)
        wimg_elems, conv_params, vec_len, stage_max = layout()
        # zero-initialised: padding rows / columns of the images must stay zero
        self.wimg = _native.zeros(wimg_elems, torch.int16, dev)
        # per-WG conv partial gradients and per-sample fc vectors (see lenet_fused.hip)
        self.slab = torch.empty((self._max_grid(), conv_params), dtype=torch.float32, device=dev)
        # (fp32 [B, 464] for the exact-fp32 kernel; the 16-bit kernels keep raw 16-bit values
        # feature-major, [464, round_up(B, 64)], in the same bytes: fc_vectors() decodes either)
        self.vslab = _native.zeros(((self.B + 63) // 64 * 64, vec_len), torch.float32, dev)
        self.loss_parts = _native.zeros(2 * self._max_grid(), torch.float32, dev)
        self.loss_acc = _native.zeros(2, torch.float32, dev)  # running (loss sum, correct)
        self.step_count = _native.zeros(1, torch.long, dev)
        self.ticket = _native.zeros(1, torch.int32, dev)
        self.cursor = _native.zeros(1, torch.long, dev)
        self.rng_offset = _native.zeros(1, torch.long, dev)
        self.eval_parts = _native.zeros(2 * 256, torch.float32, dev)
        self.perm = _native.arange(self.B, dev)
        # batch staging (per-rank batch <= stage_max): lenet_update gathers the next step's
        # pixels + labels one step ahead, so lenet_train starts with no dependent index chain
        # (the exact-fp32 kernel, lenet_fused_f32.hip, gathers its samples itself)
        self.fp32 = compute_dtype == torch.float32
        # split-K fc-gradient scratch (lenet_fused.hip fc_split_slices): per-rank batches > 1024
        # without the fused exchange form the fc weight gradients as up to 8 batch slices per
        # tile on all CUs, the tile's last slice finishing it (8 x 88 tiles x 256 partial sums,
        # then 88 arrival counters that must start at zero)
        self.fc_part = _native.zeros(8 * 88 * 256 + 128, torch.float32, dev) if self.B > 1024 else None
        # split step (lenet_fused.hip / lenet_fused_f32.hip KS > 1): split_k workgroups per sample
        # share the backward conv stages; used whenever the whole grid fits one wave of the GPU
        # (split_k * B <= 256 CUs).  CSED_SPLIT=0 keeps one workgroup per sample.  The exact-fp32
        # kernel stages its batch only in the split step.
        split_k = split_factor()
        auto = os.environ.get("CSED_SPLIT", "auto").strip().lower() != "0"
        can_stage = self.B <= stage_max and self.grid == self.B
        self.split = (can_stage and grid is None and split_k * self.B <= 256
                      and (auto if split is None else bool(split)))
        self.staged = can_stage and (not self.fp32 or self.split)
        if self.split:
            self.grid = split_k * self.B
            self.slab = torch.empty((self._max_grid(), conv_params), dtype=torch.float32, device=dev)
            self.loss_parts = _native.zeros(2 * self._max_grid(), torch.float32, dev)
        # one staging row per workgroup (split step: row r holds sample r % B)
        # the sample-tile kernel (16-bit, per-rank batch >= tile_min_batch()) stages the first tile
        # of every workgroup instead: grid * tile_samples() rows (csrc/kernels/lenet_tile.hip)
        self.tile_staged = (not self.fp32 and not self.staged and self.B >= tile_min_batch()
                            and self.grid == tile_grid(self.B))
        srows = self.grid if self.staged else (self.grid * tile_samples() if self.tile_staged else 0)
        self.xstage = _native.zeros((srows, 784), torch.uint8, dev) if srows else None
        self.lstage = _native.zeros(srows, torch.long, dev) if srows else None
        t_mark = time.perf_counter()
        self.repack()  # (the extension's first kernel launch: its code object loads here)
        self.bringup_s["first_kernel"] = time.perf_counter() - t_mark
        self._graphs: dict[tuple, object] = {}  # torch.cuda.CUDAGraph (or NativeGraph)
        self._warmed: set[str] = set()  # step kinds whose capture warm-up has run (see _capture)
        self._cap_stream: torch.cuda.Stream | None = None
        self._stepper: tuple | None = None  # (key, csed.LenetStepper), see stepper()
        self.native_max = native_max_steps()
        # which training kernel runs a step: 0 auto (the sample-tile kernel, csrc/kernels/
        # lenet_tile.hip, for 16-bit unstaged per-rank batches >= tile_min_batch()), 1 the
        # per-sample lenet_train, 2 the sample-tile kernel
        self.train_kernel = 0
        self._eval_cache: dict[int, tuple] = {}
        self._order_host: torch.Tensor | None = None
        self.capture_comm_ok: bool | None = None
        # gradient all-reduce.  Preferred: the exchange fused into lenet_update (see the module
        # docstring).  Fallback step (3 kernels: reduce-only update -> RCCL all-reduce -> SGD).
        self.exch = None
        self.exchange_note: str | None = None  # why the data-parallel step runs as it does (reports)
        self.exch_timeout_s = wait_timeout_s()
        self.path_timing_us: dict | None = None
        self._xdiag: dict = {}  # stage results of the exchange bring-up (exchange_diag)
        self._path_pending: str | None = None  # a deferred path timing (select_path)
        self.loopback_world = 0  # (set below; the exchange bring-up's reports read it)
        multi = self.comm and self.world > 1
        mode = allreduce_mode() if multi else "rccl"
        donor = reuse_exchange if (multi and reuse_exchange is not None and reuse_exchange.exch is not None
                                   and not reuse_exchange.loopback_world) else None
        if donor is not None:
            # another engine's exchange, already opened, self-tested and timed on this process
            # group (bench.py's fp32 sub-record after the 16-bit run): the IPC buffer carries
            # fp32 gradient words whatever the compute dtype, and its per-workgroup tags continue
            # on every rank alike.  The donor gives it up (its close() no longer frees it).
            self.exch, donor.exch = donor.exch, None
            self._xdiag = dict(donor._xdiag)
            self.path_timing_us = donor.path_timing_us
            self.exchange_note = "fused exchange reused from the previous engine (opened and self-tested there)"
        elif multi:
            from ..parallel.ipc import ranks_per_gpu

            self._xdiag["ranks_per_gpu"] = ranks_per_gpu(self.ctx)  # (collective: every rank)
        if donor is not None:
            pass
        elif multi and mode in ("auto", "fused"):
            self._enable_exchange(required=(mode == "fused"))
        elif multi:
            self._xdiag["ipc_open"] = f"not tried (CSED_ALLREDUCE={mode})"
        # Loopback exchange (one GPU, no process group): lenet_update runs its full push + poll
        # code for loopback_world - 1 virtual peers that are slots of this rank's own buffer
        # (csrc/comm ipc_open_loopback).  Each peer returns this rank's own gradient, and the
        # loss is scaled by 1 / (loopback_world * global batch), so the summed gradient is this
        # rank's batch mean: the same training math as world 1, at the per-step kernel cost of a
        # world-N exchange minus the xGMI flight time (the per-rank step of the driver's N-GPU
        # run, measured on one GPU: bench.py --loopback-world N).
        self.loopback_world = int(loopback_world) if loopback_world and int(loopback_world) > 1 else 0
        if self.loopback_world:
            if self.world > 1:
                raise ValueError("loopback_world is a one-GPU measurement mode (world size 1)")
            self.exch = open_loopback_exchange(self.device, exch_words(), self.loopback_world)
            self.exchange_note = f"loopback exchange: {self.loopback_world} virtual ranks on one GPU"

    @property
    def grad_scale(self) -> float:
        """Loss-gradient scale of a full step: 1 / (global batch) (x 1 / loopback_world)."""
        return 1.0 / (self.global_batch * max(1, self.loopback_world))

    # 16-bit steps run their backward at per-sample scale (dlogits = softmax - onehot, so fp16
    # gradient images stay normal numbers at any batch) and lenet_update applies the 1 / (global
    # batch) in fp32 (its grad_post); the exact-fp32 kernel takes the scale in-kernel.  For a
    # power-of-two batch both give bit-identical bf16 results.
    def _train_scale(self, grad_scale: float) -> float:
        return grad_scale if self.fp32 else 1.0

    def _post_scale(self, grad_scale: float) -> float:
        return 1.0 if self.fp32 else grad_scale

    def _vec16(self, B: int) -> torch.Tensor:
        """The 16-bit kernels' fc-vector slab of a batch of B: raw [round_up(B, 64) / 4, 464, 4]
        (sample quads, kernels/lenet_layout.h)."""
        q = (B + 63) // 64 * 16
        return self.vslab.view(-1).view(torch.int16)[:q * N_VEC * 4].view(q, N_VEC, 4)

    def fc_vectors(self, B: int | None = None) -> torch.Tensor:
        """The step's per-sample fc vectors (P2 | dZ1 | H | dlogits) as fp32 [B, 464], decoded
        from either slab layout (kernels/lenet_layout.h)."""
        B = self.B if B is None else int(B)
        if self.fp32:
            return self.vslab[:B].clone()
        v = self._vec16(B).transpose(1, 2).reshape(-1, N_VEC)[:B]  # [quad, 4, 464] -> [sample, 464]
        return v.contiguous().view(self.compute_dtype).float()

    def set_fc_vectors(self, v: torch.Tensor) -> None:
        """Fill the fc-vector slab from fp32 [B, 464] values (rounded to the compute dtype)."""
        B = v.shape[0]
        self.vslab.zero_()
        if self.fp32:
            self.vslab[:B].copy_(v)
            return
        buf = torch.zeros(((B + 63) // 64 * 64, N_VEC), dtype=self.compute_dtype, device=self.device)
        buf[:B] = v.to(device=self.device, dtype=self.compute_dtype)
        self._vec16(B).copy_(buf.view(torch.int16).view(-1, 4, N_VEC).transpose(1, 2))

    @property
    def allreduce_kind(self) -> str:
        if self.loopback_world:
            return f"fused-ipc-loopback{self.loopback_world}"
        if not self.comm:
            return "none"
        if self.exch is not None:
            return "fused-ipc"
        return "rccl"

    # ------------------------------------------------- fused gradient exchange
    def _enable_exchange(self, required: bool) -> None:
        """Bring up lenet_update's in-kernel exchange (collective on every rank): open the IPC
        buffers and self-test them with the update kernel itself.  Then (auto mode, RCCL, see
        the module docstring for ``CSED_TIME_PATHS``) the fused and fallback steps are timed
        and the faster is kept."""
        import time

        t0 = time.perf_counter()
        xd = self._xdiag
        xd["peer_access"] = _ipc.peer_access(self.device)
        ex, why = open_exchange(self.ctx, exch_words(), shared=self._xdiag.get("ranks_per_gpu"))
        hook = _ipc.test_reject_hook()
        last = self.ctx.rank == self.ctx.world_size - 1
        if hook == "open":  # (test hook: the last rank's mapping "fails"; every rank votes)
            ok_local = not last
            if not self._vote(ok_local) and ex is not None:
                ex.close()
                ex, why = None, "open: test hook CSED_TEST_EXCH_REJECT=open on the last rank"
        xd["ipc_open"] = "ok" if ex is not None else (why or "failed")
        t1 = time.perf_counter()
        self.bringup_s["ipc_open"] = t1 - t0
        ok = ex is not None
        if ok:
            self.exch = ex
            local_ok = self._exchange_self_test()
            if hook == "selftest" and last:
                local_ok = False
            xd["self_test"] = bool(local_ok)
            ok = self._vote(local_ok)
            if not ok:
                why = "self-test mismatch or timeout on some rank"
                xd["self_test_all_ranks"] = False
        self.bringup_s["self_test"] = time.perf_counter() - t1
        if not ok:
            if ex is not None:
                try:
                    ex.close()  # collective: every rank opened it (a failed rank's buffer too)
                except Exception:
                    pass
            self.exch = None
            self.exchange_note = f"fused exchange off: {why}; fallback {self.allreduce_kind}"
            if required:
                raise RuntimeError(f"CSED_ALLREDUCE=fused but the fused exchange is unusable ({why})")
            return
        self.exchange_note = "fused exchange on (self-test passed)"
        tp = os.environ.get("CSED_TIME_PATHS", "auto").strip().lower()
        if not required and tp != "0":
            # (every rank takes the same branch: ranks_per_gpu is the group's value).  On gloo
            # (ranks sharing a GPU, a rehearsal) only CSED_TIME_PATHS=1 times: the fallback step's
            # host all-reduce cannot be captured, so it times as inf and the fused path is kept --
            # what the rehearsal measures is the selection's own bring-up cost
            do_time = tp == "1" or (self.ctx.backend == "nccl" and self._xdiag.get("ranks_per_gpu") == 1)
        else:
            do_time = False
        if do_time and self.ctx.control is not None:
            # lazy RCCL (bench.py at N > 1): the fallback step's all-reduce would create the RCCL
            # communicator (1-3.6 s) in the middle of the bring-up -- the selection is deferred to
            # select_path(), which the bench runs after epoch 0 (outside the reference span)
            self._path_pending = tp
            self.exchange_note = "fused exchange on (self-test passed; path timing deferred)"
        elif do_time:
            self._select_path_now(tp)

    def select_path(self) -> bool:
        """Run the fused-vs-RCCL step timing deferred by a lazy-RCCL bring-up (collective; a no-op
        otherwise).  True if the step path changed (the cached graphs are dropped then)."""
        tp, self._path_pending = self._path_pending, None
        if tp is None or self.exch is None:
            return False
        self._select_path_now(tp)
        if self.exch is None:
            self._graphs.clear()
            self._stepper = None
            return True
        return False

    def _select_path_now(self, tp: str) -> None:
        import time

        t2 = time.perf_counter()
        t_fused = self._time_steps()
        saved, self.exch = self.exch, None
        # (gloo: the host all-reduce is not capturable -- not timed, the fused path is kept)
        t_fallback = self._time_steps() if self.ctx.backend == "nccl" else float("inf")
        t_local = float("inf")
        if tp == "1":
            # the same step with no exchange at all (each rank updates on its own gradient;
            # the state is restored): fused - local = what the exchange costs per step
            self.comm = False
            t_local = self._time_steps()
            self.comm = True
        # a path whose graph could not be captured times as inf; ties keep the fused path
        self.exch = saved if t_fused <= t_fallback else None
        if self.exch is None:
            self.exchange_note = "fused exchange off: slower than the fallback step"
            # every rank finished the timing above (device synchronize before the timing
            # all-reduce), so no peer still pushes into these buffers: the close is safe
            saved.close()
        else:
            self.exchange_note = "fused exchange on (self-test passed, timed faster than the fallback)"
        fin = lambda t: round(t, 2) if t != float("inf") else None  # noqa: E731
        self.path_timing_us = {"fused_step_us": fin(t_fused), "fallback_step_us": fin(t_fallback),
                               "local_step_us": fin(t_local),
                               "exchange_us": fin(t_fused - t_local) if max(t_fused, t_local) != float("inf")
                               else None,
                               "fallback": "rccl", "kept": "fused" if self.exch is not None else "rccl"}
        self.bringup_s["path_timing"] = time.perf_counter() - t2

    def exchange_diag(self) -> dict:
        """This rank's data-parallel diagnostics (``parallel/ipc.py`` DIAG_KEYS): the bring-up's
        stage results plus the exchange's current error word and first recorded mismatch."""
        d = _ipc.empty_diag(self.ctx)
        d.update(self._xdiag)
        d["device_count"] = torch.cuda.device_count()
        d["path_timing_us"] = self.path_timing_us
        d["allreduce"] = self.allreduce_kind
        d["note"] = self.exchange_note
        if self.exch is not None:
            d["error_word"] = self.comm_errors()
            d["first_mismatch"] = self.comm_diag()
        return d

    def _vote(self, ok: bool) -> bool:
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=_comm.ctl_device(self.ctx))
        _comm.ctl_all_reduce(self.ctx, t, dist.ReduceOp.MIN)
        return bool(t.item())

    def _exchange_self_test(self, rounds: int = 2) -> bool:
        """Integer-valued slabs through lenet_update with and without the exchange: the
        exchanged gradient must equal the process group's sum of the local ones exactly
        (both slot parities, every rank).  Runs the same collectives on every rank.  The operands
        come from the extension's own fill kernel (csed::lenet_selftest_fill: small integers, a
        hash of the element index, the round and the rank) and the results are compared on the
        host, so the bring-up launches no torch kernel (each is a code object loaded at its first
        launch, ms apiece -- the round-5 self-test drew its values with torch.randint)."""
        import numpy as np

        ops = torch.ops.csed
        pg_dev = _comm.ctl_device(self.ctx)
        common = (self.flat.data, self.momentum_buf, self.wimg, self.lr, self.momentum, self.dampening,
                  self.weight_decay, self.nesterov, self.step_count, self.ticket, None, None, False, None, 0, None,
                  self.mfma)
        ok = True
        # every round's local and exchanged gradients first, then ONE process-group all-reduce of
        # all the local ones (a collective round trip per round was most of the self-test's time)
        local = torch.empty(rounds, N_PARAMS, dtype=torch.float32, device=self.device)
        fused = torch.empty_like(local)
        for r in range(rounds):
            ops.lenet_selftest_fill(self.slab, self.vslab, self.B, self.mfma, 977 + 31 * self.ctx.rank + 7919 * r)
            ops.lenet_update(self.slab, self.grid, self.vslab, self.B, None, local[r], *common)
            try:
                ops.lenet_update(self.slab, self.grid, self.vslab, self.B, None, fused[r], *common, None,
                                 self.exch.id, self.exch_timeout_s)
            except Exception:
                ok = False
        ref = local.to(pg_dev, copy=True)
        _comm.ctl_all_reduce(self.ctx, ref)
        ok &= bool(np.array_equal(fused.cpu().numpy(), ref.cpu().numpy()))
        torch.cuda.synchronize(self.device)
        try:
            ok &= self.exch.error(reset=True) == 0
        except Exception:
            ok = False
        _native.zero_(self.vslab)
        return ok

    def _time_steps(self, nsteps: int = 16, reps: int = 3) -> float:
        """us per training step of a captured graph (max over ranks); engine state is restored."""
        state = self._state()
        saved = [t.clone() for t in state]
        try:
            g = self._capture(nsteps)
        except Exception as e:  # same code on every rank: every rank lands here
            print(f"[csed] step-graph capture failed while timing ({e!r})", file=sys.stderr)
            _clear_hip_error()
            g = None
        us = float("inf")
        if g is not None:
            g.replay()
            torch.cuda.synchronize(self.device)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                g.replay()
            b.record()
            b.synchronize()
            us = a.elapsed_time(b) * 1e3 / (reps * nsteps)
            del g
        for t, v in zip(state, saved):
            t.copy_(v)
        torch.cuda.synchronize(self.device)
        t = torch.tensor([us], dtype=torch.float64, device=_comm.ctl_device(self.ctx))
        _comm.ctl_all_reduce(self.ctx, t, dist.ReduceOp.MAX)
        return float(t.item())

    def close(self) -> None:
        """Release the graphs and the IPC buffers (collective on every rank: a barrier runs
        first so that no peer is still pushing into this rank's buffers)."""
        self._graphs.clear()
        self._stepper = None
        if self.loopback_world and self.exch is not None:  # local buffer, no peers
            torch.cuda.synchronize(self.device)
            self.exch.close()
            self.exch = None
        if self.exch is not None and dist.is_initialized():
            torch.cuda.synchronize(self.device)
            _comm.barrier(self.ctx)
        if self.exch is not None:
            self.exch.close()
        self.exch = None

    def comm_errors(self) -> int:
        """Nonzero if the IPC exchange ever timed out waiting for a peer (bit 0) or, looped back,
        received a word whose value was not the one pushed (bit 1; see ``comm_diag``).
        Synchronous."""
        return self.exch.error() if self.exch is not None else 0

    def comm_diag(self) -> dict | None:
        """The first in-kernel loopback mismatch record (block, peer row, word, tag, got, want)."""
        return self.exch.diag() if self.exch is not None else None

    def inject_exchange_fault(self, on: bool = True) -> None:
        """Fault injection (tests, ``--inject-exchange-fault``): this rank's exchange pushes go
        to a private dead-end buffer (csrc/comm ipc_set_mute), so to its peers -- or, in
        loopback mode, to itself -- it is a dead rank whose words never arrive: their waits run
        into CSED_IPC_TIMEOUT_S and raise the error word.  Captured graphs and the native
        executor hold the old mapping, so both are dropped."""
        if self.exch is None:
            raise RuntimeError("no IPC exchange to inject a fault into")
        self.exch.mute(on)
        self._graphs.clear()
        self._stepper = None

    def _max_grid(self) -> int:
        return max(self.grid, 1)

    # ----------------------------------------------------------------- state
    def repack(self) -> None:
        """Rebuild the 16-bit weight images from the fp32 master parameters."""
        torch.ops.csed.lenet_pack(self.flat.data, self.wimg, self.mfma)

    def set_epoch_order(self, order: torch.Tensor) -> None:
        """This rank's sample order for the epoch (int64 indices into the train set).

        A host order is uploaded asynchronously from pinned memory (the host never waits for
        the device here), so the next epoch's permutation can be prepared while the current
        epoch's graphs still run."""
        if order.numel() < self.B:
            raise ValueError("epoch order shorter than one batch")
        if order.device.type == "cpu":
            host = order.to(torch.long).contiguous().pin_memory()
            self._order_host = host  # alive until the copy below has run
            if host.numel() == self.perm.numel():  # straight into the captured buffer: one copy
                self.perm.copy_(host, non_blocking=True)
                _native.zero_(self.cursor)
                self._stage_current()
                return
            order = torch.empty(host.shape, dtype=torch.long, device=self.device)
            order.copy_(host, non_blocking=True)
        else:
            order = order.to(self.device, torch.long).contiguous()
        if self._graphs and order.numel() != self.perm.numel():
            self._graphs.clear()  # captured pointers refer to the old buffer
        if order.numel() == self.perm.numel():
            self.perm.copy_(order)
        else:
            self.perm = order
        _native.zero_(self.cursor)
        self._stage_current()

    def _stage_current(self) -> None:
        """Gather the batch at the cursor into the staging buffers (epoch start)."""
        if self.xstage is not None:
            torch.ops.csed.lenet_stage(self.train_data.images, self.train_data.labels, self.perm, self.cursor,
                                       self.B, self.xstage, self.lstage)



    def uses_tile_kernel(self, B: int | None = None, grid: int | None = None) -> bool:
        """Whether a full step of per-rank batch B on ``grid`` workgroups runs the sample-tile kernel
        (csrc/kernels/lenet_tile.hip) -- the launcher's own rule (bindings.cpp lenet_train) for
        kernel_for()'s choice: 16-bit, and kernel 2, or kernel 0 (auto) with B >= tile_min_batch()."""
        B = self.B if B is None else B
        grid = self.grid if grid is None else grid
        if self.fp32:
            return False
        k = self.kernel_for(B, grid)
        return k == 2 or (k == 0 and B >= tile_min_batch())

    @property
    def kernel_names(self) -> str:
        """The HIP kernels of one full training step, as launched (reports)."""
        if self.fp32:
            return "lenet_train_f32 + lenet_update"
        return ("lenet_tile" if self.uses_tile_kernel() else "lenet_train") + " + lenet_update"

    @property
    def step_kind(self) -> str:
        """How a full (staged) training step is launched."""
        return "two kernels" if (not self.comm or self.exch is not None) else "update split around an all-reduce"

    def steps_per_epoch(self) -> int:
        return math.ceil(self.perm.numel() / self.B)

    def full_steps(self) -> int:
        return self.perm.numel() // self.B

    # ------------------------------------------------------------ launches
    def _launch_step(self, B: int, grid: int, grad_scale: float, cursor: torch.Tensor | None,
                     perm: torch.Tensor) -> None:
        ops = torch.ops.csed
        # full steps read the staged batch and stage the next one; the epoch's short tail uses perm
        kern = self.kernel_for(B, grid)
        st = self._stages(kern) and cursor is not None
        ops.lenet_train(self.train_data.images, self.train_data.labels, perm, cursor, B, self.ctx.rank, self.wimg,
                        self.flat.data, self.slab, self.vslab, self.loss_parts, self._train_scale(grad_scale),
                        MNIST_MEAN, MNIST_STD, self.drop_p, self.seed, self.rng_offset, grid, self.mfma, None,
                        self.xstage if st else None, self.lstage if st else None, st, kern)
        common = (self.flat.data, self.momentum_buf, self.wimg, self.lr, self.momentum, self.dampening,
                  self.weight_decay, self.nesterov, self.step_count, self.ticket)
        post = self._post_scale(grad_scale)
        if self.exch is not None:
            ops.lenet_update(self.slab, grid, self.vslab, B, None, None, *common, cursor, self.rng_offset, True,
                             self.loss_parts, grid, self.loss_acc, self.mfma, None, self.exch.id, self.exch_timeout_s,
                             post)
        elif self.comm:
            ops.lenet_update(self.slab, grid, self.vslab, B, None, self.flat.grad, *common, None, None, False,
                             self.loss_parts, grid, self.loss_acc, self.mfma, None, -1, 2.0, post, self.fc_part)
            dist.all_reduce(self.flat.grad, op=dist.ReduceOp.SUM)
            ops.lenet_update(self.slab, grid, self.vslab, B, self.flat.grad, None, *common, cursor, self.rng_offset,
                             True, None, 0, None, self.mfma)
        else:
            ops.lenet_update(self.slab, grid, self.vslab, B, None, None, *common, cursor, self.rng_offset, True,
                             self.loss_parts, grid, self.loss_acc, self.mfma, None, -1, 2.0, post, self.fc_part)

    def _stages(self, kernel: int) -> bool:
        """Whether a full step launched with ``kernel`` (kernel_for) reads / writes the staging
        buffers: the per-sample kernel's (one row per workgroup) or the tile kernel's (first tiles)."""
        if self.staged:
            return kernel != 2
        return self.tile_staged and kernel != 1

    def kernel_for(self, B: int, grid: int) -> int:
        """``train_kernel`` for a launch of per-rank batch B on ``grid`` workgroups: the tile kernel
        only where its grid (min(256, ceil(B / tile_samples()))) is the launch's, else per-sample."""
        if self.train_kernel == 0:
            return 0 if (B < tile_min_batch() or grid == tile_grid(B)) else 1
        if self.train_kernel == 2 and grid != tile_grid(B):
            return 1
        return self.train_kernel

    def gradient(self, grid: int | None = None, dbg: torch.Tensor | None = None) -> torch.Tensor:
        """Mean-loss gradient of the batch at the cursor, without updating anything
        (lenet_train + the reduce-only lenet_update).  Also accumulates the batch's
        loss / correct count into the running totals."""
        grid = grid or self.grid
        g = torch.empty(N_PARAMS, dtype=torch.float32, device=self.device)
        ops = torch.ops.csed
        ops.lenet_train(self.train_data.images, self.train_data.labels, self.perm, self.cursor, self.B, self.ctx.rank,
                        self.wimg, self.flat.data, self.slab, self.vslab, self.loss_parts,
                        self._train_scale(1.0 / self.global_batch),
                        MNIST_MEAN, MNIST_STD, self.drop_p, self.seed, self.rng_offset, grid, self.mfma, dbg,
                        self.xstage if self._stages(self.kernel_for(self.B, grid)) and grid == self.grid else None,
                        self.lstage if self._stages(self.kernel_for(self.B, grid)) and grid == self.grid else None, False,
                        self.kernel_for(self.B, grid))
        ops.lenet_update(self.slab, grid, self.vslab, self.B, None, g, self.flat.data, self.momentum_buf, self.wimg,
                         self.lr, self.momentum, self.dampening, self.weight_decay, self.nesterov, self.step_count,
                         self.ticket, None, None, False, self.loss_parts, grid, self.loss_acc, self.mfma, None, -1,
                         2.0, self._post_scale(1.0 / self.global_batch), self.fc_part)
        return g

    def step(self) -> None:
        """One full-batch training step at the device cursor (eager launches)."""
        self._launch_step(self.B, self.grid, self.grad_scale, self.cursor, self.perm)

    def tail_size(self) -> int:
        """Per-rank samples of the epoch's short last batch (0 if the epoch divides evenly)."""
        return self.perm.numel() - self.full_steps() * self.B

    def _tail_step(self) -> None:
        rem = self.tail_size()
        tail = self.perm[self.full_steps() * self.B:]  # a view: stable pointer for graph replay
        gb = rem * self.world * max(1, self.loopback_world)  # (the sampler pads to a multiple: same on every rank)
        self._launch_step(rem, min(rem, self.grid), 1.0 / gb, None, tail)
        # the tail step does not use the cursor; keep it consistent for the next epoch
        torch.ops.csed.lenet_add_(self.cursor, 1)

    def last_partial_step(self, use_graph: bool = True) -> None:
        """The epoch's final short batch (ref DataLoader drop_last=False semantics); replayed
        from its own captured graph like the full steps."""
        if self.tail_size() <= 0:
            return
        g = self.graph(1, tail=True) if use_graph and self.capture_comm_ok is not False else None
        if g is not None:
            g.replay()
        else:
            self._tail_step()

    # --------------------------------------------------------- graph capture
    def _state(self) -> list[torch.Tensor]:
        """Device tensors a training step advances."""
        return [self.flat.data, self.momentum_buf, self.wimg, self.step_count, self.cursor, self.rng_offset,
                self.loss_acc] + ([self.xstage, self.lstage] if self.xstage is not None else [])

    def _stamp(self, key: str, dt: float) -> None:
        self.bringup_s[key] = self.bringup_s.get(key, 0.0) + dt

    def _capture(self, nsteps: int, tail: bool = False):
        """Capture ``nsteps`` full steps (or the epoch's tail step) into a HIP graph.

        The first capture of each step kind (full / tail x all-reduce path x kernel) runs one eager warm-up step on the
        capture stream first (lazy RCCL communicator set-up, each kernel's first-launch symbol
        lookup -- neither may happen inside a capture), the engine state snapshotted before and
        restored after it; later captures of the same kind skip it.  The capture calls
        capture_begin / capture_end directly: ``torch.cuda.graph``'s device synchronize and
        ``empty_cache`` are not needed (the steps allocate nothing).

        ``CSED_NATIVE_GRAPH=1`` captures a native HIP graph instead (``torch.classes.csed.HipGraph``,
        replayed by a ctypes hipGraphLaunch): it skips torch's capture_begin generator set-up (a
        torch fill kernel, ~5 ms of first-launch code-object load in the reference span), but
        measured on one box its replays start later -- 14.9-15.7 vs 14.1-14.5 us per step in the
        driver's 20-step window, 13.34 vs 13.26 us at 3000 steps (profiles/r6/graph_ab.log) -- so
        torch's graphs stay the default.  ``CSED_GRAPH_UPLOAD=1`` uploads each graph after its
        instantiation (no measured effect on the first replay).  Host seconds accumulate in
        ``bringup_s``: capture.stream / .warmup(.snapshot/.step/.sync/.restore) / .record /
        .instantiate / .upload."""
        import time

        step = self._tail_step if tail else self.step
        cur = torch.cuda.current_stream(self.device)
        t0 = time.perf_counter()
        if self._cap_stream is None:  # (one capture stream per engine: creating a stream costs ms)
            self._cap_stream = torch.cuda.Stream(self.device)
        s = self._cap_stream
        kind = f"{'tail' if tail else 'full'}/{self.allreduce_kind}/{self.train_kernel}"
        self._stamp("capture.stream", time.perf_counter() - t0)
        if kind not in self._warmed:
            # snapshot the state the capture warm-up will advance; the side stream must
            # wait for the snapshot copies too (they are enqueued on the current stream)
            ta = time.perf_counter()
            state = self._state()
            saved = [t.clone() for t in state]
            s.wait_stream(cur)
            tb = time.perf_counter()
            with torch.cuda.stream(s):
                step()
            cur.wait_stream(s)
            tc = time.perf_counter()
            torch.cuda.synchronize(self.device)
            td = time.perf_counter()
            for t, v in zip(state, saved):
                t.copy_(v)
            torch.cuda.synchronize(self.device)
            te = time.perf_counter()
            self._warmed.add(kind)
            for k, dt in (("snapshot", tb - ta), ("step", tc - tb), ("sync", td - tc), ("restore", te - td)):
                self._stamp(f"capture.warmup.{k}", dt)
        t1 = time.perf_counter()
        _comm.quiesce()  # (no pending collective for the watchdog to query during the capture)
        # thread_local: only this thread's unsafe calls invalidate the capture.  The process
        # group's watchdog thread keeps querying the events of earlier collectives while a step
        # that contains an RCCL all-reduce is captured; in the default (global) mode that query
        # invalidates the capture and the watchdog then aborts the process (seen on the GPU box,
        # profiles/round5.md)
        if os.environ.get("CSED_NATIVE_GRAPH") == "1":
            ng = torch.classes.csed.HipGraph()  # (csrc/bindings.cpp)
            with torch.cuda.stream(s):
                ng.begin(self.device.index)
                try:
                    for _ in range(nsteps):
                        step()
                finally:
                    ng.end()  # (ends the capture even after a failed step; raises if it was invalidated)
            t2 = t3 = time.perf_counter()  # (end() instantiated it)
            if os.environ.get("CSED_GRAPH_UPLOAD", "0") == "1":
                with torch.cuda.stream(cur):
                    ng.upload()
            g = NativeGraph(ng, self.device)
        else:
            g = torch.cuda.CUDAGraph(keep_graph=True)
            with torch.cuda.stream(s):
                g.capture_begin(capture_error_mode="thread_local")
                try:
                    for _ in range(nsteps):
                        step()
                finally:
                    g.capture_end()
            t2 = time.perf_counter()
            g.instantiate()
            t3 = time.perf_counter()
            if os.environ.get("CSED_GRAPH_UPLOAD", "0") == "1":
                _hip_graph_upload(g.raw_cuda_graph_exec(), cur.cuda_stream)
        t4 = time.perf_counter()
        for k, dt in (("warmup", t1 - t0), ("record", t2 - t1), ("instantiate", t3 - t2), ("upload", t4 - t3)):
            self._stamp(f"capture.{k}", dt)
        return g

    def graph(self, nsteps: int, tail: bool = False):
        """The captured graph of ``nsteps`` full steps (or of the epoch's tail step), cached."""
        key = (nsteps, self.perm.data_ptr(), self.perm.numel(), self.B, tail)
        if key in self._graphs:
            return self._graphs[key]
        if self.allreduce_kind == "rccl" and dist.is_initialized() and dist.get_backend() == "gloo":
            # the process group's all-reduce runs on the host (gloo): nothing to capture
            self.capture_comm_ok = False
            return None
        try:
            g = self._capture(nsteps, tail)
            self.capture_comm_ok = True
        except Exception as e:  # RCCL capture unsupported -> eager fallback
            print(f"[csed] HIP graph capture failed ({e!r}); running steps eagerly", file=sys.stderr)
            self.capture_comm_ok = False
            _clear_hip_error()
            torch.cuda.synchronize(self.device)
            return None
        self._graphs[key] = g
        return g

    @staticmethod
    def graph_plan(k: int, steps_per_graph: int) -> list[int]:
        """Graph sizes that run k steps: whole graphs of min(spg, k) steps, then one graph for
        the remainder (never a run of 1-step replays)."""
        if k <= 0:
            return []
        spg = max(1, min(steps_per_graph, k))
        full, rem = divmod(k, spg)
        return [spg] * full + ([rem] if rem else [])

    def prepare(self, steps_per_graph: int = 16, ks: tuple[int, ...] = (), tail: bool = True) -> None:
        """Capture up front (capture is never inside a timed region) every graph that
        ``run_steps(k, steps_per_graph)`` for k in ``ks`` (default: one epoch) and the
        epoch's tail step will replay."""
        sizes = set()
        for k in (ks or (self.full_steps(),)):
            sizes.update(self.graph_plan(k, steps_per_graph))
        for n in sorted(sizes, reverse=True):
            if self.graph(n) is None:
                return
        if tail and self.tail_size() > 0:
            self.graph(1, tail=True)

    def stepper(self):
        """The native step executor (``csrc/bindings.cpp:LenetStepper``) for this engine's full
        steps: both kernels' argument blocks built once, ``run(k)`` enqueues 2k launches from
        C++.  None where a step is more than two launches (the all-reduce fallback)."""
        if self.comm and self.exch is None:
            return None
        exch_id = -1 if self.exch is None else self.exch.id
        key = (self.perm.data_ptr(), exch_id, self.staged, self.train_kernel)
        st_ok = self._stages(self.kernel_for(self.B, self.grid))
        if self._stepper is None or self._stepper[0] != key:
            st = torch.classes.csed.LenetStepper()
            st.set_train(self.train_data.images, self.train_data.labels, self.perm, self.cursor, self.B,
                         self.ctx.rank, self.wimg, self.flat.data, self.slab, self.vslab, self.loss_parts,
                         self._train_scale(self.grad_scale), MNIST_MEAN, MNIST_STD, self.drop_p, self.seed,
                         self.rng_offset,
                         self.grid, self.mfma, self.xstage if st_ok else None,
                         self.lstage if st_ok else None, st_ok, self.kernel_for(self.B, self.grid))
            st.set_update(self.slab, self.grid, self.vslab, self.B, self.flat.data, self.momentum_buf, self.wimg,
                          self.lr, self.momentum, self.dampening, self.weight_decay, self.nesterov,
                          self.step_count, self.ticket, self.cursor, self.rng_offset, self.loss_parts, self.grid,
                          self.loss_acc, self.mfma, exch_id, self.exch_timeout_s if exch_id >= 0 else 2.0,
                          self._post_scale(self.grad_scale), self.fc_part)
            self._stepper = (key, st)
        return self._stepper[1]

    def step_plan(self, k: int, steps_per_graph: int = 16, use_graph: bool = True) -> list:
        """The launches that advance k full-batch steps from the current cursor, as a list of
        callables (graph replays, or native-executor runs where no graph applies), resolved up
        front so that a timed region holds nothing but the launches.

        Without graphs the native executor launches the steps from C++ (eager Python launches
        only where a step is more than two kernels).  Runs of at most ``self.native_max`` steps
        (``CSED_NATIVE_STEPS``, default 0) also take the executor instead of a graph replay:
        measured, graphs win even at 20 steps -- a replay's ~10 us setup is paid back by shorter
        gaps between its kernels (``profiles/bench_r2.md``, "Native step executor")."""
        if k <= 0:
            return []
        if not use_graph or self.capture_comm_ok is False or k <= self.native_max:
            st = self.stepper()
            return [self.step] * k if st is None else [lambda: st.run(k)]
        plan = []
        for n in self.graph_plan(k, steps_per_graph):
            g = self.graph(n)
            plan += [self.step] * n if g is None else [g.replay]
        return plan

    def run_steps(self, k: int, steps_per_graph: int = 16, use_graph: bool = True) -> None:
        """Advance k full-batch steps from the current cursor."""
        for launch in self.step_plan(k, steps_per_graph, use_graph):
            launch()

    def train_epoch(self, order: torch.Tensor, steps_per_graph: int = 16, use_graph: bool = True) -> None:
        self.set_epoch_order(order)
        self.run_steps(self.full_steps(), steps_per_graph, use_graph)
        self.last_partial_step(use_graph)

    # ---------------------------------------------------------------- metrics
    def take_loss(self) -> tuple[float, float]:
        """(sum of per-sample train NLL, correct count) since the last call (one host sync)."""
        v = self.loss_acc.tolist()
        self.loss_acc.zero_()
        return v[0], v[1]

    def _device_data(self, data: MNISTData) -> tuple[MNISTData, torch.Tensor]:
        """(``data`` on this engine's device, arange(len)), uploaded once per dataset object:
        evaluation runs every epoch and its 10k test images must not be re-copied each time."""
        hit = self._eval_cache.get(id(data))
        if hit is None or hit[0] is not data:
            dev = data if data.images.device == self.device else data.to(self.device)
            hit = (data, dev, _native.arange(len(data), self.device))
            self._eval_cache = {id(data): hit}
        return hit[1], hit[2]

    @torch.no_grad()
    def evaluate(self, test: MNISTData, order: torch.Tensor | None = None) -> tuple[float, int]:
        """Forward-only pass over ``test``: (summed NLL, correct).  No dropout."""
        test, ar = self._device_data(test)
        n = len(test)
        order = ar if order is None else order.to(self.device)
        nparts = min(n, 256)
        torch.ops.csed.lenet_eval(test.images, test.labels, order, n, self.wimg, self.flat.data, MNIST_MEAN,
                                  MNIST_STD, self.eval_parts, None, self.mfma)
        # (the 256 partial pairs summed on the host, in fixed order: a device reduction would be a
        # torch kernel whose code object loads at its first launch -- inside epoch 0)
        parts = self.eval_parts[: 2 * nparts].cpu().view(nparts, 2).double().sum(0).tolist()
        return parts[0], int(round(parts[1]))

    @torch.no_grad()
    def eval_logp(self, test: MNISTData) -> torch.Tensor:
        test, ar = self._device_data(test)
        n = len(test)
        out = torch.empty(n, 10, device=self.device)
        torch.ops.csed.lenet_eval(test.images, test.labels, ar, n, self.wimg,
                                  self.flat.data, MNIST_MEAN, MNIST_STD, self.eval_parts, out, self.mfma)
        return out

    # ------------------------------------------------------------ optimizer io
    def optimizer_state_dict(self) -> dict:
        """torch.optim.SGD-compatible state dict (ref results/optimizer.pth)."""
        state = {}
        if int(self.step_count.item()) > 0 and self.momentum != 0:
            for i in range(len(self.flat.params)):
                state[i] = {"momentum_buffer": self.flat.view(self.momentum_buf, i).detach().cpu().clone()}
        group = {"lr": self.lr, "momentum": self.momentum, "dampening": self.dampening,
                 "weight_decay": self.weight_decay, "nesterov": self.nesterov, "maximize": False,
                 "foreach": None, "differentiable": False, "fused": None,
                 "params": list(range(len(self.flat.params)))}
        return {"state": state, "param_groups": [group]}

    def load_optimizer_state_dict(self, sd: dict) -> None:
        have = False
        self.momentum_buf.zero_()
        for i in range(len(self.flat.params)):
            st = sd.get("state", {}).get(i)
            if st and st.get("momentum_buffer") is not None:
                self.flat.view(self.momentum_buf, i).copy_(st["momentum_buffer"])
                have = True
        self.step_count.fill_(1 if have else 0)
        g = sd["param_groups"][0]
        self.lr, self.momentum = float(g["lr"]), float(g["momentum"])
        self._graphs.clear()
        self._stepper = None  # the executor's argument blocks hold lr / momentum

    def params_changed(self) -> None:
        """Call after writing the model parameters from outside (e.g. a checkpoint load)."""
        self.repack()

    # --------------------------------------------------------------- smoke
    @classmethod
    def smoke_instance(cls, device) -> "FusedLeNetTrainer":
        from ..data.mnist import synthetic_mnist

        torch.manual_seed(1)
        net = Net().to(device)
        data = synthetic_mnist(64, seed=3)
        return cls(net, data, lr=0.01, momentum=0.5, global_batch=16)

    def smoke_step(self) -> None:
        self.set_epoch_order(torch.arange(64))
        self.step()
        torch.cuda.synchronize(self.device)
        loss, _ = self.take_loss()
        if not math.isfinite(loss):
            raise RuntimeError("fused smoke step produced a non-finite loss")
