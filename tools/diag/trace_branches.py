"""Per graph replay of graph_fork_probe.py (replays delimited by the probe's tiny add
kernels): start offset of each queue's first spin kernel after the fork and the replay's
span.  usage: trace_branches.py kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "sleep" not in r["Kernel_Name"] and "mul" not in r["Kernel_Name"].lower()]
out = []
for a, b in zip(marks, marks[1:]):
    win = rows[a + 1:b]
    if len(win) < 4:
        continue
    t0 = int(rows[a]["End_Timestamp"])
    firsts = {}
    for r in win:
        firsts.setdefault(r["Queue_Id"], int(r["Start_Timestamp"]) - t0)
    span = int(win[-1]["End_Timestamp"]) - t0
    out.append((len(win), span, firsts))
for n, span, f in out[-40:]:
    print(f"kernels {n:3d} span {span / 1e3:8.1f} us  first start per queue: "
          + ", ".join(f"q{q} +{v / 1e3:.1f}" for q, v in sorted(f.items())))
