"""Cost of a kernel boundary inside a HIP graph: N tiny dependent kernels captured once,
replayed; time per kernel (us).  Also the same with a 1024-thread x 64-block kernel."""
import torch


def per_kernel_us(fn, n=200, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / (n * reps)


def main():
    x = torch.zeros(1, device="cuda")
    y = torch.zeros(64 * 1024, device="cuda")
    print(f"tiny add (1 elem, 1 block):        {per_kernel_us(lambda: x.add_(1.0)):.2f} us/kernel")
    print(f"add over 64K floats (64+ blocks):  {per_kernel_us(lambda: y.add_(1.0)):.2f} us/kernel")


if __name__ == "__main__":
    main()
