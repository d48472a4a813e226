"""Where the step's wall time goes: busy / idle time of the GPU from a rocprofv3 kernel trace.

    python tools/trace_gaps.py gpurun_out/prof_X/bench_kernel_trace.csv [--steps N] [--marker NAME]

A step is delimited by the marker kernel (default: k_group_sumsq, the step's last pass).
For the last N steps prints the wall time, the union of kernel intervals (busy), the idle
gaps, the summed kernel time (overlap = summed - busy) and the largest gaps with the
kernels on either side.
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--marker", default="k_group_sumsq")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Stream_Id"])))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if a.marker in r[2]]
    if len(ends) < a.steps + 1:
        raise SystemExit(f"only {len(ends)} marker kernels")
    gaps_all = []
    for k in range(len(ends) - a.steps, len(ends)):
        seg = rows[ends[k - 1] + 1:ends[k] + 1]
        t0, t1 = seg[0][0], max(r[1] for r in seg)
        busy, cur_s, cur_e = 0, None, None
        gaps = []
        last_name = None
        for s, e, n, _ in seg:
            if cur_e is None:
                cur_s, cur_e, last_name = s, e, n
                continue
            if s > cur_e:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, last_name, n))
                cur_s, cur_e = s, e
            elif e > cur_e:
                cur_e = e
            if e >= cur_e:
                last_name = n
        busy += cur_e - cur_s
        summed = sum(e - s for s, e, _, _ in seg)
        wall = t1 - t0
        print(f"step {k}: wall {wall / 1e3:8.1f} us  busy {busy / 1e3:8.1f}  idle {(wall - busy) / 1e3:7.1f} "
              f"({len(gaps)} gaps)  summed {summed / 1e3:8.1f}  overlap {(summed - busy) / 1e3:7.1f}  "
              f"kernels {len(seg)} streams {sorted({r[3] for r in seg})}")
        gaps_all += gaps
    gaps_all.sort(reverse=True)
    hist = {}
    for g, _, _ in gaps_all:
        b = "<2us" if g < 2000 else "<5us" if g < 5000 else "<10us" if g < 10000 else ">=10us"
        hist[b] = hist.get(b, 0) + g
    print("idle by gap size (us, all steps):", {k: round(v / 1e3, 1) for k, v in hist.items()})
    for g, p, n in gaps_all[:a.top]:
        print(f"  gap {g / 1e3:7.1f} us after {p[:70]}  before {n[:70]}")


if __name__ == "__main__":
    main()
