"""Aggregate a rocprofv3 --pmc counter_collection.csv per kernel (mean per dispatch), then
optionally delete the raw file (it can exceed gpurun's 64 MiB copy-back limit)."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
out = sys.argv[2]
files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in files:
    with open(f) as fh:
        for r in csv.DictReader(fh):
            agg[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(out, "w") as fo:
    for k, cs in sorted(agg.items()):
        n = max(len(v) for v in cs.values())
        fo.write(f"{k} (dispatches {n})\n")
        for c, v in sorted(cs.items()):
            fo.write(f"    {c:28s} mean {sum(v) / len(v):.4g}\n")
if "--rm" in sys.argv:
    for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
        if "kernel_stats" not in f:
            os.remove(f)
