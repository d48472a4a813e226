#!/usr/bin/env python3
"""Interleaved A/B of the weight-gradient main loops on every trunk wgrad shape, in ONE
process (cdna_hip_programming.md §5.4 rule 24): k_conv_wgrad4 (mode 0) vs k_conv_wgrad_ring
(mode 1), each timed `--rounds` times alternately, the grouped launches the step runs (both
views per launch), operands rotating over more than the 256 MiB Infinity Cache.

    python tools/wgrad_ab.py [--batch 64] [--rounds 3] [--reps 10] [--arch resnet18]
"""
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
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--groups", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--modes", default="0,1")
    a = ap.parse_args()
    import trunk_table as T
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import build
    build.build()
    dev = torch.device("cuda:0")
    lib = L.load()
    modes = [int(m) for m in a.modes.split(",")]
    ops = [o for o in T.conv_ops(a.batch, dev, 320e6, a.groups, a.arch) if o[1] == "wgrad"]
    res = {(name, m): [] for name, *_ in ops for m in modes}
    for _ in range(a.rounds):
        for m in modes:
            L.check(lib.gm_conv_set_wgrad_ring(m), "ring")
            for name, op, cnt, flops, nbytes, fn in ops:
                res[(name, m)].append(T._time(fn, a.reps))
    L.check(lib.gm_conv_set_wgrad_ring(0), "ring")
    tot = {m: [0.0, 0.0] for m in modes}
    print(f"| shape | x/step | GFLOP | " + " | ".join(f"mode {m} us (TF/s, frac)" for m in modes) + " |")
    print("|---|---|---|" + "---|" * len(modes))
    for name, op, cnt, flops, nbytes, fn in ops:
        cells = []
        for m in modes:
            t = statistics.median(res[(name, m)])
            tot[m][0] += flops * cnt
            tot[m][1] += t * cnt
            cells.append(f"{t * 1e6:.1f} ({flops / t / 1e12:.0f}, {flops / t / 1e12 / 2500:.3f})")
        print(f"| {name} | {cnt} | {flops / 1e9:.2f} | " + " | ".join(cells) + " |")
    for m in modes:
        fl, s = tot[m]
        print(f"mode {m}: wgrad family {fl / 1e12:.3f} TFLOP in {s * 1e3:.3f} ms = {fl / s / 1e12:.1f} TF/s = "
              f"{fl / s / 1e12 / 2500:.3f} of 2500", flush=True)


if __name__ == "__main__":
    main()
