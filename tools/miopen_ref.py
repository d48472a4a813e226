"""Calibration: the same ResNet-18 trunk convolutions through PyTorch-ROCm's own library
path (MIOpen, bf16, channels_last, autotuned with cudnn.benchmark) at the step's batch (both
views: 2 x 64 images), forward / input gradient / weight gradient, HIP-event timed.  Not a
product path - a yardstick for tools/trunk_table.py's rows.

    python tools/miopen_ref.py [--batch 128] [--reps 20]
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import trunk_table as T
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda:0")
    B = a.batch
    print(f"| shape | pass | GFLOP | MIOpen us | TFLOP/s |\n|---|---|---|---|---|")
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    flops_tot = 0.0
    for name, (C, H, W, K, R, st, pad, cnt) in T.TRUNK:
        P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
        x = torch.randn(B, C, H, W, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = torch.randn(K, C, R, R, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        dy = torch.randn(B, K, P, Q, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        flops = 2.0 * B * P * Q * K * C * R * R
        ops = {
            "fwd": lambda: F.conv2d(x, w, stride=st, padding=pad),
            "dgrad": lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [st, st], [pad, pad], [1, 1], False,
                                                                 [0, 0], 1, [True, False, False]),
            "wgrad": lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [st, st], [pad, pad], [1, 1], False,
                                                                 [0, 0], 1, [False, True, False]),
        }
        for p, op in ops.items():
            for _ in range(3):
                op()
            t = T._time(op, a.reps)
            tot[p] += t * cnt
            flops_tot += flops * cnt
            print(f"| {name} | {p} | {flops / 1e9:.2f} | {t * 1e6:.1f} | {flops / t / 1e12:.1f} |", flush=True)
    s = sum(tot.values())
    print(f"\nMIOpen trunk convolutions: fwd {tot['fwd'] * 1e3:.3f} ms, dgrad {tot['dgrad'] * 1e3:.3f} ms, "
          f"wgrad {tot['wgrad'] * 1e3:.3f} ms; total {s * 1e3:.3f} ms = {flops_tot / s / 1e12:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
