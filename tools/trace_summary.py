"""Per (kernel, grid) mean duration from a rocprofv3 kernel_trace.csv."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if pat not in n:
        continue
    g = (r.get("Grid_Size_X", r.get("Grid_Size", "?")), r.get("Grid_Size_Y", ""))
    agg[(n[:60], g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (n, g), v in sorted(agg.items()):
    print(f"{n:60s} grid={g} n={len(v)} mean_us={sum(v) / len(v):.2f} min_us={min(v):.2f}")
