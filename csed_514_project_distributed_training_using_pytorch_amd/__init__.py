"""MI355X-native data-parallel CNN training framework.

A brand-new implementation of the capabilities of
abhishekiitm/CSED_514_Project_Distributed_Training_using_PyTorch (MNIST `Net`,
single-process and DDP trainers, point-to-point smoke test) for AMD MI355X
(gfx950): hand-written HIP/CDNA4 kernels (MFMA + LDS) for every op, a fused
two-launch training step replayed from HIP graphs, RCCL over xGMI for data
parallelism.

Subpackages: ``ops`` (kernel library), ``models`` (Net + layers), ``optim``
(fused SGD), ``parallel`` (process groups, DDP reducer, sampler, launcher),
``data`` (MNIST IDX/synthetic + device loader), ``engine`` (fused / modular
trainers, CLI), ``utils`` (checkpoints, metrics, plots, profiling).
"""
__version__ = "0.1.0"

from . import data, models, ops, optim, parallel, utils  # noqa: F401
