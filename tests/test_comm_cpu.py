"""CPU-side pieces of the data-parallel gradient exchange (parallel/ipc.py, engine/fused.py).

The exchange itself runs in HIP kernels and is covered on a GPU by tests/test_comm_gpu.py;
here: mode selection, the collective-safe bring-up returning "unusable" off-GPU, and the
exchange buffer layout the update kernel and the host agree on.
"""
import pytest
import torch

from csed_514_project_distributed_training_using_pytorch_amd.parallel import ipc
from csed_514_project_distributed_training_using_pytorch_amd.parallel.comm import DistContext


@pytest.mark.parametrize("value,mode", [(None, "auto"), ("auto", "auto"), ("FUSED", "fused"), ("rccl", "rccl")])
def test_allreduce_mode(monkeypatch, value, mode):
    if value is None:
        monkeypatch.delenv("CSED_ALLREDUCE", raising=False)
    else:
        monkeypatch.setenv("CSED_ALLREDUCE", value)
    assert ipc.allreduce_mode() == mode


@pytest.mark.parametrize("value", ["nvlink", "ipc"])
def test_allreduce_mode_rejects_unknown(monkeypatch, value):
    # "ipc" (the one-shot kernel as a training path) was removed in round 4: only gradient paths
    # with a strict test remain selectable
    monkeypatch.setenv("CSED_ALLREDUCE", value)
    with pytest.raises(ValueError):
        ipc.allreduce_mode()


def test_make_allreduce_mode_checked():
    single = DistContext(0, 1, 0, torch.device("cpu"), None)
    with pytest.raises(ValueError):
        ipc.make_allreduce(single, 21840, mode="fused")


def test_no_ipc_without_distributed_gpu(monkeypatch):
    monkeypatch.delenv("CSED_ALLREDUCE", raising=False)
    single = DistContext(0, 1, 0, torch.device("cpu"), None)
    assert ipc.make_allreduce(single, 21840) is None
    ex, why = ipc.open_exchange(single, 27840)
    assert ex is None and why
    # a gloo (CPU) group of two: still no IPC buffers (they are device memory)
    cpu_pair = DistContext(0, 2, 0, torch.device("cpu"), "gloo")
    assert ipc.make_allreduce(cpu_pair, 21840) is None
    assert ipc.open_exchange(cpu_pair, 27840)[0] is None


def test_exchange_buffer_layout():
    """lenet_update's exchange words: the conv slab slots 0..5375 (one word each), each of the
    88 fc tiles owns 256 words after the conv slab row (csrc/kernels/lenet_layout.h: conv1's
    260 slots padded to 5 chunks, conv2's 5020 to 79: 84 chunks of 64 = 5376)."""
    from csed_514_project_distributed_training_using_pytorch_amd.ops import _native

    if not _native.load(build_if_missing=False):
        pytest.skip("native extension not built")
    layout = [int(v) for v in torch.ops.csed.lenet_layout()]
    conv_pad, nparams, words = layout[1], layout[3], layout[5]
    assert nparams == 21840 and conv_pad == 5376 and layout[6] == 4  # split step: 4 workgroups / sample
    assert len(layout) == 9 and layout[7] == 4 and layout[8] == 1024  # sample tiles of 4 from batch 1024
    fc_tiles = 4 * 21 + 4  # fc1: 4 x 21 tiles of [dW1 | db1], fc2: 4 tiles of [dW2 | db2]
    assert words == conv_pad + fc_tiles * 256 == 27904
    assert words % 4 == 0  # the IPC buffers are allocated in multiples of 4 words
