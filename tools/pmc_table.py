"""Summarise rocprofv3 --pmc counter_collection.csv files per (kernel, grid size):
mean counter value per dispatch, dispatch count.  usage: pmc_table.py <dir>"""
import collections
import csv
import glob
import os
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            key = (r["Kernel_Name"][:100], r.get("Grid_Size", "?"), r.get("Workgroup_Size", "?"))
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (k, grid, wg), cs in sorted(agg.items()):
    n = max(len(v) for v in cs.values())
    vals = "  ".join(f"{c}={sum(v) / len(v):.6g}" for c, v in sorted(cs.items()))
    print(f"{k} | grid {grid} wg {wg} | n {n} | {vals}")
