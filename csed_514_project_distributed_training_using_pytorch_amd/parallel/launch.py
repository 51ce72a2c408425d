"""Local multi-process launcher: one process per MI355X (replaces the reference's
"start the script by hand on every VM" with hard-coded ranks, ref src/train_dist.py:118-146,
src/run1.py:27-37).

    python -m csed_514_project_distributed_training_using_pytorch_amd.parallel.launch \\
        --nproc 8 [--master-addr 127.0.0.1] [--master-port 29500] script.py [script args...]

Each child gets the torchrun environment contract (RANK, LOCAL_RANK, WORLD_SIZE,
LOCAL_WORLD_SIZE, MASTER_ADDR, MASTER_PORT) and ``--local_rank`` is NOT
appended (scripts read the environment).  Children are started as separate
processes (never exec'd from a GPU-initialised parent).  The first non-zero
exit terminates the remaining ranks and is returned (fail fast instead of
the reference's wait-for-timeout).
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def free_port(addr: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((addr, 0))
        return s.getsockname()[1]


def launch(nproc: int, cmd: list[str], master_addr: str = "127.0.0.1", master_port: int | None = None,
           env_extra: dict | None = None, timeout: float | None = None) -> int:
    port = master_port or free_port(master_addr)
    procs = []
    for r in range(nproc):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(nproc), "LOCAL_WORLD_SIZE": str(nproc),
                    "MASTER_ADDR": master_addr, "MASTER_PORT": str(port)})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if env_extra:
            env.update(env_extra)
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
    t0 = time.time()
    rc = 0
    try:
        while True:
            alive = 0
            for p in procs:
                code = p.poll()
                if code is None:
                    alive += 1
                elif code != 0 and rc == 0:
                    rc = code
            if rc != 0 or alive == 0:
                break
            if timeout is not None and time.time() - t0 > timeout:
                rc = 124
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
    return rc


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nproc", "--nproc-per-node", type=int, default=1)
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=None)
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = [sys.executable, a.script, *a.args]
    return launch(a.nproc, cmd, a.master_addr, a.master_port, timeout=a.timeout)


if __name__ == "__main__":
    sys.exit(main())
