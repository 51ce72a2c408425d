"""The native build's rebuild decision is by content (_build.py): a source whose bytes change
is rebuilt even when its mtime is older than its object, and an untouched source is not."""
import os

from csed_514_project_distributed_training_using_pytorch_amd import _build


def test_stamp_follows_content_not_mtime(tmp_path):
    src = tmp_path / "k.hip"
    obj = tmp_path / "k.o"
    src.write_text("__global__ void k() {}\n")
    cmd = ["hipcc", "-O3", "-c", str(src), "-o", str(obj)]
    st = _build._src_stamp(src, "hdr", cmd)
    obj.write_bytes(b"obj")
    obj.with_suffix(".tag").write_text(st)
    assert not _build._needs(obj, st)
    # new content, old mtime (older than the object): must rebuild
    old = obj.stat().st_mtime - 100
    src.write_text("__global__ void k() { int x = 1; (void)x; }\n")
    os.utime(src, (old, old))
    st2 = _build._src_stamp(src, "hdr", cmd)
    assert st2 != st and _build._needs(obj, st2)
    # a header change or a flag change also changes the stamp
    assert _build._src_stamp(src, "hdr2", cmd) != st2
    assert _build._src_stamp(src, "hdr", cmd + ["-g"]) != st2
    # same content touched newer: no rebuild
    obj.with_suffix(".tag").write_text(st2)
    os.utime(src, None)
    assert not _build._needs(obj, _build._src_stamp(src, "hdr", cmd))
