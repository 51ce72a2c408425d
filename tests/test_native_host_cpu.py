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


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_synth_generator_under_host_sanitizers(tmp_path):
    """csrc/data/synth_mnist.cpp under ASan + UBSan: the bilinear resampler's taps stay inside the
    bordered source image for every sample, and the sanitized build produces exactly
    the production library's bytes."""
    import numpy as np

    from csed_514_project_distributed_training_using_pytorch_amd.data import native_synth

    exe = tmp_path / "synth_check"
    cmd = [HIPCC, "-O1", "-g", "-std=c++17", "-fno-gpu-sanitize", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-pthread", os.path.join(ROOT, "tests", "native", "synth_check.cpp"),
           os.path.join(ROOT, "csrc", "data", "synth_mnist.cpp"), "-o", str(exe)]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stderr[-3000:]
    protos = np.ascontiguousarray(native_synth.prototypes(10), dtype=np.float32)
    pf, out = tmp_path / "protos.bin", tmp_path / "out.bin"
    protos.tofile(pf)
    n = 3000
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), str(pf), str(n), str(out)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    raw = np.fromfile(out, dtype=np.uint8)
    images = raw[: n * 784].reshape(n, 28, 28)
    labels = raw[n * 784:].view(np.int64)
    if native_synth.available():
        ref_img, ref_lab = native_synth.generate(n, seed=7, train=True)
        assert np.array_equal(np.asarray(ref_img).reshape(n, 28, 28), images)
        assert np.array_equal(np.asarray(ref_lab), labels)
