"""The strided first convolutions of layers 2-4 (k_conv_igemm_ut: l2.0.c1 / l3.0.c1 / l4.0.c1,
forward and input gradient) as the step launches them (both views per grouped launch, B = 64 per
view): main-loop form (gm_conv_set_pipe 0 / 2 / 3) x split-K target (gm_conv_set_splitk), one
process, interleaved rounds, HIP events:

    python tools/diag/strided_ab.py [--rounds 5]
"""
import argparse
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ds", action="store_true")
    a = ap.parse_args()
    import trunk_table as T
    from greedy_multimodal_learning_amd import _lib as L
    lib = L.load()
    dev = torch.device("cuda:0")
    trunk = dict(T.TRUNKS["resnet18"])
    arms = [(0, 384), (2, 384), (3, 384), (0, 0), (0, 768)]
    if "--ds" in sys.argv:  # the 1x1 / s2 downsamples: the main-loop form only
        arms = [(0, 384), (2, 384)]
    for name in (("l2.ds", "l3.ds", "l4.ds") if "--ds" in sys.argv else ("l2.0.c1", "l3.0.c1", "l4.0.c1")):
        C, H, W, K, R, st, pad, cnt = trunk[name]
        P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
        for op in ("fwd", "dgrad"):
            fn = T._make_bf16(op, 64, dev, C, H, W, K, R, st, pad, P, Q, 2)
            flops = 2.0 * 2 * 64 * P * Q * K * C * R * R
            t = {arm: [] for arm in arms}
            for _ in range(a.rounds):
                for arm in arms:
                    L.check(lib.gm_conv_set_pipe(arm[0]), "pipe")
                    L.check(lib.gm_conv_set_splitk(arm[1]), "splitk")
                    t[arm].append(T._time(fn, a.reps))
            L.check(lib.gm_conv_set_pipe(-1), "pipe")
            L.check(lib.gm_conv_set_splitk(384), "splitk")
            print(f"{name} {op:5s}: " + "  ".join(
                f"pipe {p} splitk {s}: {statistics.median(v) * 1e6:6.1f} us ({flops / statistics.median(v) / 2.5e15:.3f})"
                for (p, s), v in t.items()), flush=True)


if __name__ == "__main__":
    main()
