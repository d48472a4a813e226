"""Run ONE trunk convolution shape repeatedly (for rocprofv3 --pmc passes):

    python tools/conv_one.py --shape l2 --op fwd --pipe 0 --reps 50
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

CL = torch.channels_last


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="l2")
    ap.add_argument("--op", default="fwd", choices=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--groups", type=int, default=2, help="wgrad: views per grouped launch")
    ap.add_argument("--ring", type=int, default=None, help="wgrad: gm_conv_set_wgrad_loop mode")
    ap.add_argument("--pipe", type=int, default=-1)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--sets", type=int, default=1, help="grouped stem/wgrad: distinct operand sets cycled")
    a = ap.parse_args()
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import conv as G
    import trunk_table as T
    dev = torch.device("cuda:0")
    C, H, W, K, R, st, pad, _ = dict(T.TRUNK)[a.shape]
    B = a.batch
    P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
    x = torch.randn(B, C, H, W, device=dev).bfloat16().contiguous(memory_format=CL)
    w = torch.randn(K, C, R, R, device=dev).bfloat16().contiguous(memory_format=CL)
    dy = torch.randn(B, K, P, Q, device=dev).bfloat16().contiguous(memory_format=CL)
    wt = w.permute(1, 0, 2, 3).contiguous(memory_format=CL)
    L.check(L.load().gm_conv_set_pipe(a.pipe), "set_pipe")
    fn = (lambda: G.conv_fwd(x, w, st, pad)) if a.op == "fwd" else (lambda: G.conv_dgrad_t(dy, wt, H, W, st, pad))
    if a.shape == "conv1" and a.op == "fwd":  # the pixel-pair stem, grouped as in the step
        fns = [T._make_bf16("fwd", B, dev, C, H, W, K, R, st, pad, P, Q, a.groups) for _ in range(a.sets)]
        fn = fns[0] if a.sets == 1 else T._cycle(fns)
        B = B * a.groups
    if a.op == "wgrad":  # the step's grouped launch (both views), as tools/trunk_table.py builds it
        if a.ring is not None:
            L.check(L.load().gm_conv_set_wgrad_loop(a.ring), "ring")
        fn = T._make_bf16("wgrad", B, dev, C, H, W, K, R, st, pad, P, Q, a.groups)
        B = B * a.groups
    t = T._time(fn, a.reps)
    flops = 2.0 * B * P * Q * K * C * R * R
    print(f"{a.shape} {a.op} pipe {a.pipe}: {t * 1e6:.2f} us, {flops / t / 1e12:.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
