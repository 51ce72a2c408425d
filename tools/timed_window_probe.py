"""Fixed cost of a short timed window (bench.py's driver command times 20 steps between two
host synchronisations): wall-clock (sync; replay; sync) per plan of graphs, against the
device-event time of the same replays.  Prints us per window and us per step."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from csed_514_project_distributed_training_using_pytorch_amd.data import synthetic_mnist  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.engine.fused import FusedLeNetTrainer  # noqa: E402
from csed_514_project_distributed_training_using_pytorch_amd.models import Net  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    dev = torch.device("cuda")
    data = synthetic_mnist(64 * 256, seed=1)  # 256 steps at B = 64: every plan stays inside the order
    torch.manual_seed(1)
    eng = FusedLeNetTrainer(Net().to(dev), data, global_batch=B)
    eng.set_epoch_order(torch.randperm(len(data)))
    plans = {"1": [1], "2": [2], "5": [5], "20": [20], "1+19": [1, 19], "2+18": [2, 18], "4+16": [4, 16],
             "200": [200], "19": [19], "18": [18], "16": [16]}
    for p in plans.values():
        for n in p:
            eng.graph(n)
    eng.step()
    res = {}
    plans.update({"sleep+1": ["s", 1], "sleep+20": ["s", 20], "eager1": ["e"], "eager5": ["e"] * 5, "eager20": ["e"] * 20,
                  "native1": [("n", 1)], "native5": [("n", 5)], "native20": [("n", 20)], "native200": [("n", 200)],
                  "sleep+native20": ["s", ("n", 20)],
                  # the first step(s) from the native executor, the rest as one graph replay: does the
                  # graph's launch latency hide behind the native steps?
                  "n1+19": [("n", 1), 19], "n2+18": [("n", 2), 18], "n4+16": [("n", 4), 16]})
    st = eng.stepper()  # csed.LenetStepper: the native step executor
    st.run(1)
    for name, p in plans.items():
        walls, evs = [], []
        for _ in range(30):
            eng.cursor.zero_()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            if p[0] == "s":  # keep the GPU busy while the host submits what follows
                torch.cuda._sleep(200000)
            a.record()
            for n in p:
                if n == "e":
                    eng.step()
                elif isinstance(n, tuple):
                    st.run(n[1])
                elif n != "s":
                    eng.graph(n).replay()
            b.record()
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e6)
            evs.append(a.elapsed_time(b) * 1e3)
        walls.sort()
        evs.sort()
        k = sum(1 if n == "e" else n[1] if isinstance(n, tuple) else n for n in p if n != "s")
        res[name] = (walls[15], evs[15])
        print(f"B={B} plan {name:5s}: wall {walls[15]:8.1f} us ({walls[15] / k:6.2f}/step)   "
              f"events {evs[15]:8.1f} us ({evs[15] / k:6.2f}/step)", flush=True)


if __name__ == "__main__":
    main()
