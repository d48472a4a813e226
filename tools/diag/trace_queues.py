"""First launches of the last N kernels of a rocprofv3 kernel_trace.csv, per queue, as
offsets from the first of them (graph_fork_probe.py).  usage: trace_queues.py csv N"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-int(sys.argv[2]):]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:8.1f} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:6.1f}"
          f" q{r['Queue_Id']} {r['Kernel_Name'][:60]}")
