"""Interleaved A/B of the weight-gradient kernel choice (gm_conv_set_wgrad_loop modes) on the
view-batched trunk's grouped launches (G = 2 views, B = 64 per view), split sums included:

    python tools/wgrad_ab.py [--modes 6,22] [--rounds 5] [--arch resnet18] [--shapes l3,l4]

Per shape and mode: median and min of the per-round average launch time (HIP events), TFLOP/s
and the fraction of the 2.5 PF dense bf16 peak."""
import argparse
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="6:22")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--groups", type=int, default=2)
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--shapes", default="l2.0.c1,l2,l3.0.c1,l3,l4.0.c1,l4")
    a = ap.parse_args()
    import trunk_table as T
    from greedy_multimodal_learning_amd import _lib as L
    lib = L.load()
    dev = torch.device("cuda:0")
    # a mode is a gm_conv_set_wgrad_loop value
    modes = a.modes.replace(":", ",").split(",")

    def set_mode(m):
        L.check(lib.gm_conv_set_wgrad_loop(int(m)), "loop")
    trunk = dict(T.TRUNKS[a.arch])
    B, G = a.batch, a.groups
    print(f"{a.arch} wgrad, G={G}, B={B}, modes {modes}, {a.rounds} rounds x {a.reps} reps", flush=True)
    tot = {m: 0.0 for m in modes}
    flops_tot = 0.0
    for name in a.shapes.replace(":", ",").split(","):
        C, H, W, K, R, st, pad, cnt = trunk[name]
        P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
        fn = T._make_bf16("wgrad", B, dev, C, H, W, K, R, st, pad, P, Q, G)
        flops = 2.0 * G * B * P * Q * K * C * R * R
        times = {m: [] for m in modes}
        for _ in range(a.rounds):
            for m in modes:
                set_mode(m)
                times[m].append(T._time(fn, a.reps))
        parts = []
        for m in modes:
            med, mn = statistics.median(times[m]), min(times[m])
            tot[m] += med * cnt
            parts.append(f"mode {m:>4s}: {med * 1e6:7.1f} us (min {mn * 1e6:6.1f}) {flops / med / 1e12:6.1f} TF/s "
                         f"{flops / med / 2.5e15:.3f}")
        flops_tot += flops * cnt
        print(f"{name:8s} x{cnt}  " + " | ".join(parts), flush=True)
    print("per step (x count): " + " | ".join(f"mode {m}: {tot[m] * 1e6:.1f} us = {flops_tot / tot[m] / 2.5e15:.3f}"
                                               for m in modes), flush=True)
    set_mode("22")


if __name__ == "__main__":
    main()
