"""Relative L2 error of the fused 16-bit gradients against the fp32 CPU Net (dropout off), per
parameter, for the per-sample kernel (B = 64) and the tile kernel (B = 1024), bf16 and fp16.
Usage: python tools/grad_bands.py"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist
from csed_514_project_distributed_training_using_pytorch_amd.data.mnist import MNIST_MEAN, MNIST_STD
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer
from csed_514_project_distributed_training_using_pytorch_amd.models import Net

DEV = torch.device("cuda")


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm()).item()


for B in (64, 1024, 8192):
    data = synthetic_mnist(max(2048, B), seed=11)
    order = torch.randperm(max(2048, B), generator=torch.Generator().manual_seed(0))[:B]
    for dt in (torch.bfloat16, torch.float16):
        torch.manual_seed(1)
        net, ref = Net(), Net()
        ref.load_state_dict(net.state_dict())
        eng = FusedLeNetTrainer(net.to(DEV), data, global_batch=B, compute_dtype=dt, drop_p=0.0)
        eng.set_epoch_order(order)
        g = eng.gradient().cpu()
        # the same batch with the round-1..3 scaling: 1 / B inside the 16-bit backward
        kern = eng.kernel_for(B, eng.grid)
        st = eng._stages(kern)
        ops = torch.ops.csed
        ops.lenet_train(eng.train_data.images, eng.train_data.labels, eng.perm, eng.cursor, B, 0, eng.wimg,
                        eng.flat.data, eng.slab, eng.vslab, eng.loss_parts, 1.0 / B, MNIST_MEAN, MNIST_STD, 0.0,
                        eng.seed, eng.rng_offset, eng.grid, eng.mfma, None, eng.xstage if st else None,
                        eng.lstage if st else None, False, kern)
        g_pre = torch.empty_like(eng.flat.data)
        ops.lenet_update(eng.slab, eng.grid, eng.vslab, B, None, g_pre, eng.flat.data, eng.momentum_buf, eng.wimg,
                         eng.lr, eng.momentum, eng.dampening, eng.weight_decay, eng.nesterov, eng.step_count,
                         eng.ticket, None, None, False, None, 0, None, eng.mfma)
        g_pre = g_pre.cpu()
        x = ((data.images[order].float() / 255.0 - MNIST_MEAN) / MNIST_STD).to(dt).float().view(-1, 1, 28, 28)
        ref.eval()
        F.nll_loss(ref(x), data.labels[order]).backward()
        off, out = 0, []
        for name, p in ref.named_parameters():
            n = p.numel()
            out.append(f"{name} {rel(g[off:off + n].view_as(p), p.grad):.2e} (1/B in-kernel {rel(g_pre[off:off + n].view_as(p), p.grad):.2e})")
            off += n
        print(f"B={B} {str(dt)[6:]:9s} kernel={'tile' if eng.kernel_for(B, eng.grid) == 0 and B >= 1024 else 'per-sample'}: " + ", ".join(out), flush=True)
