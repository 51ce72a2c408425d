"""Build driver for the native extension (`_C.so`).

Everything under ``csrc/`` is compiled with ``hipcc --offload-arch=gfx950``
directly -- no hipify pass, no CUDA sources, no JIT cache.  The resulting
shared object lives next to this file so it travels with the repository
snapshot to the GPU box and is found by :func:`load`.

Layout of the native code:

* ``csrc/kernels/*.hip`` -- device kernels plus plain-pointer launchers.  These
  translation units do not include any torch header, so they compile in a few
  seconds each.
* ``csrc/bindings.cpp`` -- the only TU that sees ATen: tensor checks, stream
  lookup and ``TORCH_LIBRARY`` registration of the ``csed::*`` ops.

Usage::

    python -m csed_514_project_distributed_training_using_pytorch_amd._build [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO = PKG_DIR.parent
CSRC = REPO / "csrc"
BUILD_DIR = REPO / "build" / "native"
SO_PATH = PKG_DIR / "_C.so"
ARCH = os.environ.get("CSED_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the native extension needs ROCm's hipcc")


def _torch_flags() -> tuple[list[str], list[str]]:
    import torch
    import torch.utils.cpp_extension as ce

    inc = []
    for p in ce.include_paths():
        inc += ["-isystem", p]
    inc += ["-isystem", sysconfig.get_paths()["include"]]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    defs = [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1"]
    torch_lib = str(Path(torch.__file__).parent / "lib")
    libs = [
        f"-L{torch_lib}",
        f"-Wl,-rpath,{torch_lib}",
        "-lc10",
        "-lc10_hip",
        "-ltorch_cpu",
        "-ltorch_hip",
        "-ltorch",
    ]
    return inc + defs, libs


COMMON = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result",
          "-munsafe-fp-atomics"]


def _sources() -> tuple[list[Path], list[Path]]:
    kernels = sorted((CSRC / "kernels").glob("*.hip")) + sorted((CSRC / "comm").glob("*.hip"))
    hosts = sorted(CSRC.glob("*.cpp"))
    return kernels, hosts


def _headers_digest() -> str:
    h = hashlib.sha1()
    for p in sorted(CSRC.rglob("*.h")):
        h.update(p.read_bytes())
    return h.hexdigest()[:12]


def _src_stamp(src: Path, common: str, cmd: list[str]) -> str:
    """Content stamp of one object: the source's bytes, every header's bytes (``common``) and
    the compile command (flags, arch).  Modification times play no part, so a source whose
    content changed is rebuilt even when its mtime is older than its object (a checkout, a
    copy with preserved times), and an untouched source is not rebuilt after a ``touch``."""
    h = hashlib.sha1()
    h.update(src.read_bytes())
    h.update(common.encode())
    h.update("\0".join(c for c in cmd if c not in (str(src),)).encode())
    return h.hexdigest()


def _needs(obj: Path, stamp: str) -> bool:
    tag = obj.with_suffix(".tag")
    if not obj.exists() or not tag.exists():
        return True
    return tag.read_text() != stamp


def _compile(cmd: list[str], obj: Path, stamp: str) -> str:
    obj.with_suffix(".tag").unlink(missing_ok=True)  # (a failed compile leaves no valid stamp)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    obj.with_suffix(".tag").write_text(stamp)
    return obj.name


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> Path:
    """Compile every HIP/C++ source for gfx950 and link ``_C.so`` in-tree."""
    hipcc = _hipcc()
    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    tflags, tlibs = _torch_flags()
    kernels, hosts = _sources()
    common = _headers_digest() + ARCH
    jobs = jobs or min(8, os.cpu_count() or 4, 16)
    cmds = []
    objs = []
    stamps = []
    for src in kernels + hosts:
        obj = BUILD_DIR / (src.stem + ".o")
        objs.append(obj)
        if src in kernels:
            cmd = [hipcc, *COMMON, f"-I{CSRC}", "-c", str(src), "-o", str(obj)]
        else:
            cmd = [hipcc, *COMMON, *tflags, f"-I{CSRC}", "-x", "hip", "-c", str(src), "-o", str(obj)]
        stamp = _src_stamp(src, common, cmd)
        stamps.append(stamp)
        if force or _needs(obj, stamp):
            cmds.append((cmd, obj, stamp))
    # the shared object's own stamp: every object's stamp, so a relink follows any rebuilt object
    so_stamp = hashlib.sha1("".join(stamps).encode()).hexdigest()
    so_tag = SO_PATH.with_suffix(".tag")
    if cmds:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = [ex.submit(_compile, c, o, st) for c, o, st in cmds]
            for f in cf.as_completed(futs):
                name = f.result()
                if verbose:
                    print(f"[csed build] compiled {name}", flush=True)
    link_needed = (force or bool(cmds) or not SO_PATH.exists() or not so_tag.exists()
                   or so_tag.read_text() != so_stamp)
    if link_needed:
        tmp = SO_PATH.with_suffix(".so.tmp")
        cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), *tlibs,
               "-o", str(tmp)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, SO_PATH)
        so_tag.write_text(so_stamp)
        if verbose:
            print(f"[csed build] linked {SO_PATH}", flush=True)
    return SO_PATH


DATA_SO = PKG_DIR / "_csed_data.so"


def build_data_lib(force: bool = False, verbose: bool = True) -> Path:
    """Host-only native data generator (``csrc/data/synth_mnist.cpp`` -> ``_csed_data.so``):
    plain g++, no torch and no HIP, so it loads before ``import torch``."""
    src = CSRC / "data" / "synth_mnist.cpp"
    cxx = os.environ.get("CXX") or shutil.which("g++") or shutil.which("c++")
    if not cxx:
        raise RuntimeError("no host C++ compiler for the data generator")
    tmp = DATA_SO.with_suffix(".so.tmp")
    cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-ffp-contract=off", "-march=x86-64-v2", str(src), "-o", str(tmp)]
    stamp = _src_stamp(src, "", cmd)
    tag = DATA_SO.with_suffix(".tag")
    if not force and DATA_SO.exists() and tag.exists() and tag.read_text() == stamp:
        return DATA_SO
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, DATA_SO)
    tag.write_text(stamp)
    if verbose:
        print(f"[csed build] built {DATA_SO}", flush=True)
    return DATA_SO


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs)
    build_data_lib(force=a.force)
    return 0


if __name__ == "__main__":
    sys.exit(main())
