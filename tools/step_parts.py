"""Where a bench step's wall time goes: full steps (replay + eager tail + host gate
sync) vs bare back-to-back graph replays of the same captured step."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    from greedy_multimodal_learning_amd.engine import BalancedStep
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = MMTM_MVCNN().to(dev)
    gate = Bias_Mitigation_Strong(epsilon=0.01, curation_windowsize=5, branchnames=["net_view_0", "net_view_1"],
                                  starting_epoch=1)
    st = BalancedStep(m, lr=0.1, gate=gate, graphs=True)
    st.on_epoch_begin(1)
    g = torch.Generator(device=dev).manual_seed(1000)
    B = 64
    x = torch.randn(2, B, 224, 224, 3, device=dev, generator=g).bfloat16().permute(1, 0, 4, 2, 3)
    y = torch.randint(0, 40, (B,), device=dev, generator=g)
    for _ in range(6):
        st(x, y)
    torch.cuda.synchronize()
    n = 30
    t0 = time.perf_counter()
    for _ in range(n):
        st(x, y)
    torch.cuda.synchronize()
    full = (time.perf_counter() - t0) / n * 1e3
    gr = next(iter(st._graphs.values()))[0]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        gr.replay()
    torch.cuda.synchronize()
    rep = (time.perf_counter() - t0) / n * 1e3
    print(f"full step {full:.3f} ms, bare graph replay {rep:.3f} ms, host/tail {full - rep:.3f} ms", flush=True)
    # CPU cost of the launch call itself: one replay enqueued on an idle GPU, timed to return
    cpu = []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gr.replay()
        cpu.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
    cpu.sort()
    # back-to-back: does a launch call wait for the previous replay of the same graph?
    torch.cuda.synchronize()
    ts = [time.perf_counter()]
    for _ in range(8):
        gr.replay()
        ts.append(time.perf_counter())
    torch.cuda.synchronize()
    te = time.perf_counter()
    print("back-to-back launch calls (ms): " + " ".join(f"{(b - a) * 1e3:.2f}" for a, b in zip(ts, ts[1:]))
          + f"; then sync {(te - ts[-1]) * 1e3:.2f}", flush=True)
    print(f"graph launch call (CPU, returns before the GPU finishes): median {cpu[5] * 1e3:.3f} ms, "
          f"min {cpu[0] * 1e3:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
