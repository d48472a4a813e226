"""One bench step as a kernel listing from a rocprofv3 kernel_trace.csv: every launch of
the median step (steps delimited by the fused norms+SGD launch k_group_sumsq<true>) in
start order with its offset, duration, queue and grid, plus the step's concurrency
profile (time with 0 / 1 / 2 / 3+ kernels running) and the busy time per kernel family
split by how many other kernels ran beside it.

    python tools/step_listing.py kernel_trace.csv [--list]
"""
import csv
import re
import sys


def family(name):
    n = name
    for pat, fam in (("k_conv_halo", "conv_halo"), ("k_conv_rw", "conv_rw"), ("k_conv_stem", "conv_stem"),
                     ("k_conv_igemm", "conv_igemm"), ("k_conv_wgrad", "wgrad"), ("k_wgrad_sum", "wgrad_sum"),
                     ("k_bn_bwd", "bn_bwd"), ("k_bn_fwd", "bn_fwd"), ("k_bn_", "bn_other"), ("maxpool", "maxpool"),
                     ("k_gemm_f32", "gemm_f32"), ("copyBuffer", "copy"), ("group_sumsq", "sgd"),
                     ("k_weight_prep", "wprep"), ("k_wprep", "wprep"), ("k_colreduce", "mmtm"),
                     ("k_channel_scale", "mmtm"), ("k_rowreduce", "mmtm"), ("xent", "loss")):
        if pat in n:
            return fam
    return re.sub(r"^(void )?(gm::)?(\(anonymous namespace\)::)?", "", n).split("(")[0].split("<")[0][:24]


def main():
    path = sys.argv[1]
    listing = "--list" in sys.argv
    rows = list(csv.DictReader(open(path)))
    ks = []
    for r in rows:
        q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
        grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], q, grid))
    ks.sort()
    marks = [i for i, k in enumerate(ks) if "k_group_sumsq<true" in k[2]]
    wins = [(a, b) for a, b in zip(marks, marks[1:]) if b > a + 1]
    if not wins:
        print("no complete step window")
        return
    wins.sort(key=lambda w: ks[w[1]][1] - ks[w[0]][1])
    a, b = wins[len(wins) // 2]
    win = ks[a + 1:b + 1]
    t0 = ks[a][1]
    t1 = win[-1][1]
    print(f"median step: {len(win)} kernels, wall {(t1 - t0) / 1e3:.1f} us")
    # concurrency profile over [t0, t1]
    ev = []
    for s, e, n, q, g in win:
        ev.append((max(s, t0), 1, n))
        ev.append((e, -1, n))
    ev.sort(key=lambda x: (x[0], x[1]))
    hist = {}
    cur, last = 0, t0
    running = []
    fam_alone = {}
    fam_shared = {}
    for t, d, n in ev:
        if t > last:
            k = min(cur, 3)
            hist[k] = hist.get(k, 0) + (t - last)
            for rn in running:
                tgt = fam_alone if cur == 1 else fam_shared
                tgt[family(rn)] = tgt.get(family(rn), 0) + (t - last) / cur
            last = t
        cur += d
        if d > 0:
            running.append(n)
        else:
            running.remove(n)
    tot = sum(hist.values())
    print("concurrency: " + "  ".join(f"{k if k < 3 else '3+'}: {v / 1e3:.1f} us ({v / tot:.0%})"
                                       for k, v in sorted(hist.items())))
    fams = sorted(set(fam_alone) | set(fam_shared), key=lambda f: -(fam_alone.get(f, 0) + fam_shared.get(f, 0)))
    print("family     alone(us)  shared-share(us)")
    for f in fams:
        print(f"{f:12s} {fam_alone.get(f, 0) / 1e3:8.1f} {fam_shared.get(f, 0) / 1e3:10.1f}")
    if listing:
        for s, e, n, q, g in win:
            print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{q:>3s} g{g:>8s} {n[:90]}")


if __name__ == "__main__":
    main()
