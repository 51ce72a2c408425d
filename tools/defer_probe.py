#!/usr/bin/env python3
"""Per-parameter gradient difference of Net's backward with the weight-gradient reduce deferred /
carried vs not (diagnostics for ops.set_defer_wgrad_reduce)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch

    from csed_514_project_distributed_training_using_pytorch_amd import ops
    from csed_514_project_distributed_training_using_pytorch_amd.models import Net
    from csed_514_project_distributed_training_using_pytorch_amd.ops import functional as fn

    torch.manual_seed(1)
    net = Net().cuda().train()
    g = torch.Generator(device="cuda").manual_seed(13)
    x = torch.rand(64, 1, 28, 28, device="cuda", generator=g)
    t = torch.randint(0, 10, (64,), device="cuda", generator=g)
    res = {}
    for mode in ("fused-defer", "fused-nodefer", "logp-defer", "logp-nodefer"):
        fn.set_defer_wgrad_reduce(mode.endswith("-defer"))
        ops.rng.default_state.reset_offset()
        net.zero_grad(set_to_none=True)
        loss = net(x, target=t) if mode.startswith("fused") else ops.nll_loss(net(x), t)
        loss.backward()
        torch.cuda.synchronize()
        print(mode, "pending after backward:", fn.pending_reduce_count())
        res[mode] = {n: p.grad.clone() for n, p in net.named_parameters()}
    for a, b in (("fused-defer", "fused-nodefer"), ("logp-defer", "logp-nodefer"), ("fused-nodefer", "logp-nodefer")):
        print(a, "vs", b, {n: round((res[a][n] - res[b][n]).abs().max().item(), 6) for n in res[a]})
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
