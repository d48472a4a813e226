#!/usr/bin/env python3
"""Interleaved A/B of a convolution kernel knob (a gm_conv_set_* setter of the library) on
the trunk shapes, in ONE process (cdna_hip_programming.md §5.4 rule 24): every mode timed
`--rounds` times alternately on the grouped launches the step runs (both views per launch),
operands rotating over more than the 256 MiB Infinity Cache.

    python tools/conv_knob_ab.py --setter gm_conv_set_wgrad_loop --modes 0,6 --ops wgrad --shapes l1,l2
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
    ap.add_argument("--setter", default="gm_conv_set_wgrad_loop")
    ap.add_argument("--ops", default="wgrad", help="comma list of fwd, dgrad, wgrad")
    ap.add_argument("--shapes", default="", help="comma list of trunk shape names (default all)")
    ap.add_argument("--default", type=int, default=None, help="mode restored at the end (default: first)")
    a = ap.parse_args()
    import trunk_table as T
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import build
    build.build()
    dev = torch.device("cuda:0")
    lib = L.load()
    modes = [int(m) for m in a.modes.replace("/", ",").split(",")]
    want_ops = set(a.ops.replace("/", ",").split(","))
    want_shapes = set(a.shapes.replace("/", ",").split(",")) if a.shapes else None
    ops = [o for o in T.conv_ops(a.batch, dev, 320e6, a.groups, a.arch)
           if o[1] in want_ops and (want_shapes is None or o[0] in want_shapes)]
    setter = getattr(lib, a.setter)
    res = {(name, op, m): [] for name, op, *_ in ops for m in modes}
    for _ in range(a.rounds):
        for m in modes:
            L.check(setter(m), a.setter)
            for name, op, cnt, flops, nbytes, fn in ops:
                res[(name, op, m)].append(T._time(fn, a.reps))
    L.check(setter(modes[0] if a.default is None else a.default), a.setter)
    tot = {m: [0.0, 0.0] for m in modes}
    print(f"{a.setter}: modes {modes}, ops {a.ops}, batch {a.batch} x {a.groups} views, {a.rounds} rounds (median)")
    print(f"| shape | pass | x/step | GFLOP | " + " | ".join(f"mode {m} us (TF/s, frac)" for m in modes) + " |")
    print("|---|---|---|---|" + "---|" * len(modes))
    for name, op, cnt, flops, nbytes, fn in ops:
        cells = []
        for m in modes:
            t = statistics.median(res[(name, op, m)])
            tot[m][0] += flops * cnt
            tot[m][1] += t * cnt
            cells.append(f"{t * 1e6:.1f} ({flops / t / 1e12:.0f}, {flops / t / 1e12 / 2500:.3f})")
        print(f"| {name} | {op} | {cnt} | {flops / 1e9:.2f} | " + " | ".join(cells) + " |")
    for m in modes:
        fl, s = tot[m]
        print(f"mode {m}: these launches {fl / 1e12:.3f} TFLOP in {s * 1e3:.3f} ms = {fl / s / 1e12:.1f} TF/s = "
              f"{fl / s / 1e12 / 2500:.3f} of 2500", flush=True)


if __name__ == "__main__":
    main()
