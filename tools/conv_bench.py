"""Per-shape timing of the trunk convolutions (own MFMA kernels vs MIOpen), B=64, one view."""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from greedy_multimodal_learning_amd import conv as G  # noqa: E402

SHAPES = {  # name: (N, C, H, W, K, R, S, stride, pad, count per view)
    "conv1": (64, 3, 224, 224, 64, 7, 7, 2, 3, 1),
    "l1": (64, 64, 56, 56, 64, 3, 3, 1, 1, 4),
    "l2.0.c1": (64, 64, 56, 56, 128, 3, 3, 2, 1, 1),
    "l2.ds": (64, 64, 56, 56, 128, 1, 1, 2, 0, 1),
    "l2": (64, 128, 28, 28, 128, 3, 3, 1, 1, 3),
    "l3.0.c1": (64, 128, 28, 28, 256, 3, 3, 2, 1, 1),
    "l3.ds": (64, 128, 28, 28, 256, 1, 1, 2, 0, 1),
    "l3": (64, 256, 14, 14, 256, 3, 3, 1, 1, 3),
    "l4.0.c1": (64, 256, 14, 14, 512, 3, 3, 2, 1, 1),
    "l4.ds": (64, 256, 14, 14, 512, 1, 1, 2, 0, 1),
    "l4": (64, 512, 7, 7, 512, 3, 3, 1, 1, 3),
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
    return e0.elapsed_time(e1) / it * 1e3  # us


def main():
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = True
    only = sys.argv[1:] or list(SHAPES)
    tot = {"own": 0.0, "miopen": 0.0}
    print(f"{'shape':9s} {'op':6s} {'own_us':>8s} {'TF/s':>7s} {'miopen_us':>9s} {'TF/s':>7s}")
    for name in only:
        N, C, H, W, K, R, S, st, pad, cnt = SHAPES[name]
        P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - S) // st + 1
        flops = 2.0 * N * P * Q * K * C * R * S
        Cp = G._cpad(C)
        x = torch.randn(N, Cp, H, W, device=dev).bfloat16().contiguous(memory_format=G.CL)
        w = torch.randn(K, Cp, R, S, device=dev).bfloat16().contiguous(memory_format=G.CL)
        dy = torch.randn(N, K, P, Q, device=dev).bfloat16().contiguous(memory_format=G.CL)
        xm, wm = x[:, :C].contiguous(memory_format=G.CL), w[:, :C].contiguous(memory_format=G.CL)
        ops = {
            "fwd": (lambda: G.conv_fwd(x, w, st, pad),
                    lambda: F.conv2d(xm, wm, stride=st, padding=pad)),
            "dgrad": (lambda: G.conv_dgrad(dy, w, H, W, st, pad),
                      lambda: torch.ops.aten.convolution_backward(dy, xm, wm, None, [st, st], [pad, pad], [1, 1],
                                                                  False, [0, 0], 1, [True, False, False])),
            "wgrad": (lambda: G.conv_wgrad(dy, x, R, S, st, pad, C),
                      lambda: torch.ops.aten.convolution_backward(dy, xm, wm, None, [st, st], [pad, pad], [1, 1],
                                                                  False, [0, 0], 1, [False, True, False])),
        }
        for op, (own, mio) in ops.items():
            if name == "conv1" and op == "dgrad":
                continue
            if os.environ.get("CB_OPS") and op not in os.environ["CB_OPS"].split(","):
                continue
            t_own = timeit(own)
            t_mio = timeit(mio) if not os.environ.get("CB_NOMIO") else 1e9
            tot["own"] += t_own * cnt
            tot["miopen"] += t_mio * cnt
            print(f"{name:9s} {op:6s} {t_own:8.1f} {flops / t_own / 1e6:7.1f} {t_mio:9.1f} {flops / t_mio / 1e6:7.1f}",
                  flush=True)
    print(f"per-view trunk conv total: own {tot['own'] / 1e3:.3f} ms, miopen {tot['miopen'] / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
