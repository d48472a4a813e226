"""Step timeline from a rocprofv3 kernel_trace.csv: steps are delimited by the
per-step k_group_sumsq<true> (fused norms + SGD) launch.  For each step window
prints the wall time, the union of kernel-busy time (GPU idle = wall - union),
the summed kernel time (overlap = sum / union) and the longest idle gaps with
the kernels either side.  usage: python tools/timeline.py kernel_trace.csv [n_gaps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ngap = int(sys.argv[2]) if len(sys.argv) > 2 else 8
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
marks = [i for i, k in enumerate(ks) if "k_group_sumsq<true>" in k[2]]
steps = []
for a, b in zip(marks, marks[1:]):
    win = ks[a + 1:b + 1]
    if not win:
        continue
    t0, t1 = ks[a][1], win[-1][1]
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    prev_name = ks[a][2]
    cur_e = t0
    for s, e, n in win:
        if s > cur_e:
            gaps.append((s - cur_e, prev_name[:50], n[:50]))
        if e > cur_e:
            busy += e - max(s, cur_e)
            cur_e = e
            prev_name = n
    tot = sum(e - s for s, e, _ in win)
    steps.append((t1 - t0, busy, tot, len(win), sorted(gaps, reverse=True)[:ngap]))
for w, u, t, n, _ in steps:
    print(f"step wall {w / 1e3:8.1f} us  busy {u / 1e3:8.1f}  idle {(w - u) / 1e3:7.1f}  kernels {n:4d}  "
          f"sum {t / 1e3:8.1f}  overlap {t / max(u, 1):.2f}")
if steps:
    mid = sorted(steps, key=lambda s: s[0])[len(steps) // 2]
    print("largest idle gaps of the median step:")
    for g, p, n in mid[4]:
        print(f"  {g / 1e3:7.1f} us  after {p}  before {n}")
