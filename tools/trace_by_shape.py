"""Per-(kernel, grid, VGPR/LDS) duration table from a rocprofv3 kernel_trace.csv.

usage: python tools/trace_by_shape.py <kernel_trace.csv> [name-substring ...]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    subs = sys.argv[2:]
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(list)
    meta = {}
    for r in rows:
        name = r["Kernel_Name"]
        if subs and not any(s in name for s in subs):
            continue
        grid = (int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), int(r["Grid_Size_Y"]),
                int(r["Grid_Size_Z"]))
        key = (name[:70], grid)
        agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        meta[key] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"], r["Scratch_Size"])
    tot = sum(sum(v) for v in agg.values())
    print(f"{'us_total':>9s} {'n':>5s} {'avg':>8s} {'min':>8s}  vgpr/agpr/lds/scr  grid  name")
    for key, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        m = meta[key]
        print(f"{sum(v):9.1f} {len(v):5d} {sum(v) / len(v):8.2f} {min(v):8.2f}  {m[0]}/{m[1]}/{m[2]}/{m[3]}  "
              f"{key[1]}  {key[0]}")
    print(f"total {tot:.1f} us")


if __name__ == "__main__":
    main()
