"""A/B of the implicit-GEMM conv kernel's forms: main loop (gm_conv_set_pipe 0 / 2 / 3;
5 / 6 timing diagnostics) and the halo kernel for 3x3/s1 (gm_conv_set_halo; variant
"h" = halo on, pipe 0)
on every ResNet-18 trunk shape of one view (fwd + dgrad), interleaved rounds in ONE
process (cdna_hip_programming.md §5.4 rule 24), HIP events behind a device sleep.
Also checks that every variant's outputs are bitwise equal to variant 0's (same
reduction order: only the staging schedule differs).

    python tools/conv_ab.py [--batch 64] [--rounds 5] [--pipes 0,2,3]
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
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--pipes", default="0,h", help="comma list of pipe numbers; 'h' = halo kernel on (k_conv_h9), "
                                                 "'o' = halo kernel with run-time tap decode, 'H' = 256-pixel halo tiles")
    ap.add_argument("--wgrad", action="store_true", help="also time the weight-gradient passes")
    ap.add_argument("--shapes", default="", help="'+'-separated trunk shape names (default: all)")
    a = ap.parse_args()
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import conv as G
    import trunk_table as T
    dev = torch.device("cuda:0")
    B = a.batch
    pipes = a.pipes.replace("+", ",").split(",")

    def select(p):  # "h": the halo kernel; "H...": 256-pixel halo tiles;
        # "o": the halo kernel with run-time tap decode (k_conv_halo) instead of k_conv_h9;
        # "fBN.NB": k_conv_h9 forced to BN-channel tiles and an NB-stage weight ring
        # "s<n>": split-K target n (0: never split), auto form otherwise
        L.check(lib.gm_conv_set_splitk(int(p[1:]) if p[0] == "s" else 384), "set_splitk")
        # "g<n>": weight-gradient operand staging n (gm_conv_set_wgrad_staging)
        L.check(lib.gm_conv_set_wgrad_staging(int(p[1:]) if p[0] == "g" else 0), "set_wgrad_staging")
        if p[0] == "g":
            p = "h"
        if p[0] == "s":
            p = "h"
        if p[0] == "f":
            bn, nb = p[1:].split(".")
            L.check(lib.gm_conv_set_h9((int(bn) << 8) | int(nb)), "set_h9")
        else:
            L.check(lib.gm_conv_set_h9(0 if p == "o" else 1), "set_h9")
        if p[0] in ("W", "o", "f"):
            p = "h"
        hl = p[:1] in ("h", "H")
        L.check(lib.gm_conv_set_halo((2 if p[0] == "H" else 1) if hl else 0), "set_halo")
        L.check(lib.gm_conv_set_pipe(int(p[1:] or 0) if hl else int(p)), "set_pipe")
    lib = L.load()
    ops = []
    g = torch.Generator(device=dev).manual_seed(0)
    only = set(a.shapes.split("+")) if a.shapes else None
    for name, (C, H, W, K, R, st, pad, cnt) in T.TRUNK:
        if C == 3 or (only and name not in only):
            continue
        P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
        flops = 2.0 * B * P * Q * K * C * R * R
        x = torch.randn(B, C, H, W, device=dev, generator=g).bfloat16().contiguous(memory_format=CL)
        w = torch.randn(K, C, R, R, device=dev, generator=g).bfloat16().contiguous(memory_format=CL)
        dy = torch.randn(B, K, P, Q, device=dev, generator=g).bfloat16().contiguous(memory_format=CL)
        wt = w.permute(1, 0, 2, 3).contiguous(memory_format=CL)
        ops.append((name, "fwd", cnt, flops, (lambda x=x, w=w, st=st, pad=pad: G.conv_fwd(x, w, st, pad))))
        ops.append((name, "dgrad", cnt, flops,
                    (lambda dy=dy, wt=wt, H=H, W=W, st=st, pad=pad: G.conv_dgrad_t(dy, wt, H, W, st, pad))))
        if a.wgrad:
            dw = torch.empty(K, C, R, R, device=dev, dtype=torch.float32).contiguous(memory_format=CL)
            ops.append((name, "wgrad", cnt, flops,
                        (lambda dy=dy, x=x, R=R, st=st, pad=pad, C=C, dw=dw: G.conv_wgrad(dy, x, R, R, st, pad, C,
                                                                                          out=dw))))
    # correctness: pipe variants == variant 0 bitwise; the halo kernel (another
    # summation order) within bf16 output rounding of it
    ref = {}
    for p in pipes:
        if p in ("5", "6", "h5", "h6", "H5", "H6", "h7", "h8"):
            continue  # timing diagnostics: outputs meaningless
        select(p)
        for name, op, _, _, fn in ops:
            out = fn()
            torch.cuda.synchronize()
            k = (name, op)
            if k not in ref:
                ref[k] = out.clone()
                continue
            d = (out.float() - ref[k].float()).abs().max().item()
            sc = ref[k].float().abs().max().item()
            if (p[:1] not in ("h", "H", "W", "o", "f", "s", "r", "g") and not torch.equal(out, ref[k])) or d > 2e-2 * sc:
                print(f"MISMATCH {p} {name} {op}: max |diff| {d} (scale {sc})", flush=True)
                sys.exit(3)
    print("all variants agree", flush=True)
    times = {(p, n, o): [] for p in pipes for n, o, *_ in ops}
    for r in range(a.rounds):
        for p in pipes:
            select(p)
            for name, op, _, _, fn in ops:
                times[(p, name, op)].append(T._time(fn, a.reps))
        print(f"round {r} done", flush=True)
    print(f"| shape | pass | " + " | ".join(f"{p} us (TF/s)" for p in pipes) + " |")
    tot = {p: [0.0, 0.0] for p in pipes}
    for name, op, cnt, flops, _ in ops:
        cells = []
        for p in pipes:
            ts = sorted(times[(p, name, op)])
            t = ts[len(ts) // 2]
            tot[p][0] += flops * cnt
            tot[p][1] += t * cnt
            cells.append(f"{t * 1e6:.1f} ({flops / t / 1e12:.0f})")
        print(f"| {name} | {op} | " + " | ".join(cells) + " |")
    for p in pipes:
        print(f"{p}: family {tot[p][0] / tot[p][1] / 1e12:.1f} TFLOP/s "
              f"({tot[p][1] * 1e3:.3f} ms per view)")
    select("h")


if __name__ == "__main__":
    main()
