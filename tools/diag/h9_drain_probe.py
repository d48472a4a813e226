"""k_conv_h9 with and without its per-chunk halo reload (gm_conv_set_pipe(7): the next chunk's
halo is NOT loaded - outputs meaningless, timing only), grouped launches as the step runs them:

    python tools/diag/h9_drain_probe.py [--rounds 5]
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
    a = ap.parse_args()
    import trunk_table as T
    from greedy_multimodal_learning_amd import _lib as L
    lib = L.load()
    dev = torch.device("cuda:0")
    trunk = dict(T.TRUNKS["resnet18"])
    for name in ("l2", "l3", "l4"):
        C, H, W, K, R, st, pad, cnt = trunk[name]
        P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
        for op in ("fwd", "dgrad"):
            fn = T._make_bf16(op, 64, dev, C, H, W, K, R, st, pad, P, Q, 2)
            flops = 2.0 * 2 * 64 * P * Q * K * C * R * R
            t = {0: [], 7: []}
            for _ in range(a.rounds):
                for p in (0, 7):
                    L.check(lib.gm_conv_set_pipe(p), "pipe")
                    t[p].append(T._time(fn, a.reps))
            L.check(lib.gm_conv_set_pipe(0), "pipe")
            m0, m7 = statistics.median(t[0]), statistics.median(t[7])
            print(f"{name} {op:5s}: with halo reload {m0 * 1e6:6.1f} us ({flops / m0 / 2.5e15:.3f})  without "
                  f"{m7 * 1e6:6.1f} us ({flops / m7 / 2.5e15:.3f})", flush=True)


if __name__ == "__main__":
    main()
