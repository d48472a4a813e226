"""Per-shape timing of the fused BatchNorm(+add+ReLU) kernels vs PyTorch/MIOpen, B=64."""
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from greedy_multimodal_learning_amd.bn import GMBatchNorm2d  # noqa: E402

CL = torch.channels_last
SHAPES = {  # name: (N, C, H, W, residual, count per view)
    "stem": (64, 64, 112, 112, False, 1),
    "l1": (64, 64, 56, 56, True, 4),
    "l2": (64, 128, 28, 28, True, 5),
    "l3": (64, 256, 14, 14, True, 5),
    "l4": (64, 512, 7, 7, True, 5),
}


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    dev = torch.device("cuda:0")
    tot = {"own": 0.0, "torch": 0.0}
    print(f"{'shape':6s} {'own_us':>8s} {'GB/s':>7s} {'torch_us':>9s}")
    for name, (N, C, H, W, res, cnt) in SHAPES.items():
        x = torch.randn(N, C, H, W, device=dev).bfloat16().contiguous(memory_format=CL).requires_grad_(True)
        r = torch.randn(N, C, H, W, device=dev).bfloat16().contiguous(memory_format=CL) if res else None
        dy = torch.randn(N, C, H, W, device=dev).bfloat16().contiguous(memory_format=CL)
        own = GMBatchNorm2d(C).to(dev)
        ref = nn.BatchNorm2d(C).to(dev)

        def f_own():
            y = own(x, residual=r, relu=True)
            y.backward(dy)

        def f_ref():
            y = ref(x)
            if r is not None:
                y = y + r
            F.relu(y).backward(dy)

        t_own, t_ref = timeit(f_own), timeit(f_ref)
        # algorithmic bytes: fwd x(2) + x,r,y (2+2+2) ; bwd dy,y,x (6) + dy,y,x,dx(,dres) (8/10)
        eb = 2 + (6 if res else 4) + 6 + (10 if res else 8)
        gbs = N * C * H * W * eb / t_own / 1e3
        tot["own"] += t_own * cnt
        tot["torch"] += t_ref * cnt
        print(f"{name:6s} {t_own:8.1f} {gbs:7.0f} {t_ref:9.1f}", flush=True)
    print(f"per-view BN fwd+bwd total: own {tot['own'] / 1e3:.3f} ms, torch {tot['torch'] / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
