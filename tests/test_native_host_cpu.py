"""Host-side sanitizer build (race / memory-error detection): the fused kernels'
slab layout (csrc/kernels/lenet_layout.h) compiled for the host with AddressSanitizer and
UndefinedBehaviorSanitizer and checked to be a one-to-one map onto the slab buffer for every
grid / batch the kernels use.  (GPU sanitizers are not available on this pool; the layout is
what decides whether two workgroups' slab writes could collide or leave the buffer.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_slab_layout_under_host_sanitizers(tmp_path):
    exe = tmp_path / "layout_check"
    cmd = [HIPCC, "-O1", "-g", "-std=c++17", "-fno-gpu-sanitize", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", f"-I{os.path.join(ROOT, 'csrc')}",
           os.path.join(ROOT, "tests", "native", "layout_check.cpp"), "-o", str(exe)]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "layout check ok" in r.stdout
