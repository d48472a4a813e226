"""Per-op hardware counters of the trunk launches (tools/trunk_table.py ops), for
rocprofv3 --pmc passes.  `run` mode (under the profiler): each op is preceded by a
marker (torch.cuda._sleep -> `spin_kernel`) and called R times, so the counter rows
between two markers belong to R calls of one op.  `report` mode: join the passes'
counter_collection.csv files into a per-op table:

  HBM bytes per call  = 2 x FETCH_SIZE + WRITE_SIZE (KB = 1024 B; FETCH_SIZE doubled:
                        gfx950 reports half of wide streaming reads, MI355X_MICROARCH.md)
  MFMA busy           = SQ_VALU_MFMA_BUSY_CYCLES / (32 x SQ_BUSY_CYCLES) (SQ_BUSY_CYCLES
                        sums the 32 shader engines of 32 SIMDs each: the fraction of
                        SIMD-cycles with the matrix pipe busy during the op's dispatches)

    rocprofv3 --pmc FETCH_SIZE -d out/fetch -o pmc -- python3 tools/trunk_pmc.py run
    python3 tools/trunk_pmc.py report out/fetch out/write out/mfma [--json conv.json] > table.md
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
R = 4


def run():
    import torch
    import trunk_table as T
    dev = torch.device("cuda:0")
    ops = T.conv_ops(64, dev) + T.bn_ops(64, dev)
    for _ in ops:  # warm every op once (kernel attributes, workspaces)
        pass
    for name, op, cnt, flops, nbytes, fn in ops:
        fn()
    torch.cuda.synchronize()
    for name, op, cnt, flops, nbytes, fn in ops:
        torch.cuda._sleep(1000)
        for _ in range(R):
            fn()
        torch.cuda.synchronize()
    with open(os.path.join(ROOT, "gpurun_out", "trunk_pmc_ops.json"), "w") as f:
        json.dump([dict(name=n, op=o, count=c, flops=fl, bytes=b) for n, o, c, fl, b, _ in ops], f)


def _segments(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    by = {}
    for r in rows:
        k = int(r["Dispatch_Id"])
        by.setdefault(k, [r["Kernel_Name"], {}])[1][r["Counter_Name"]] = float(r["Counter_Value"])
    segs, cur, started = [], None, False
    for k in sorted(by):
        kname, cs = by[k]
        if "spin_kernel" in kname:
            if cur is not None:
                segs.append(cur)
            cur = {"kernels": set(), "n": 0, "c": {}}
            continue
        if cur is None:
            continue  # warm-up calls before the first marker
        cur["kernels"].add(kname.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:60])
        cur["n"] += 1
        for c, v in cs.items():
            cur["c"][c] = cur["c"].get(c, 0.0) + v
    if cur is not None:
        segs.append(cur)
    return segs


def report(dirs, json_out=None):
    ops = json.load(open(os.path.join(ROOT, "gpurun_out", "trunk_pmc_ops.json")))
    seg_sets = [_segments(d) for d in dirs]
    rows = []
    for i, o in enumerate(ops):
        c = {}
        kern, nd = set(), 0
        for segs in seg_sets:
            if i < len(segs):
                c.update(segs[i]["c"])
                kern |= segs[i]["kernels"]
                nd = segs[i]["n"]
        fetch = c.get("FETCH_SIZE", float("nan")) * 1024 * 2 / R
        write = c.get("WRITE_SIZE", float("nan")) * 1024 / R
        busy = c.get("SQ_BUSY_CYCLES")
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
        util = mf / (32 * busy) if busy and mf is not None else float("nan")
        lds_c = c.get("SQ_LDS_BANK_CONFLICT", float("nan")) / R
        rows.append(dict(o, kernels=sorted(kern), dispatches_per_call=nd // R if nd else 0, hbm_read=fetch,
                         hbm_write=write, mfma_busy=util, lds_bank_conflict_cycles=lds_c,
                         insts_mfma=c.get("SQ_INSTS_MFMA", float("nan")) / R,
                         insts_lds=c.get("SQ_INSTS_LDS", float("nan")) / R))
    print("| shape | pass | kernels | HBM MB/call (PMC) | algorithmic MB | ratio | MFMA busy | LDS bank-conflict cycles |")
    print("|---|---|---|---|---|---|---|---|")
    for r in rows:
        t = r["hbm_read"] + r["hbm_write"]
        print(f"| {r['name']} | {r['op']} | {', '.join(k.split('::')[-1][:28] for k in r['kernels'])} | "
              f"{t / 1e6:.1f} | {r['bytes'] / 1e6:.1f} | {t / r['bytes']:.2f} | {r['mfma_busy']:.3f} | "
              f"{r['lds_bank_conflict_cycles']:.3g} |")
    conv = [r for r in rows if r["flops"]]
    w = sum(r["count"] for r in conv)
    fam = {
        "what": "trunk convolution family as the step launches it: both views per launch (view-batched trunk), "
                "B=64 per view (fwd + dgrad + wgrad of every position, count-weighted as bench.py's roofline), "
                "HBM bytes from rocprofv3 PMC (2 x FETCH_SIZE + WRITE_SIZE per call)",
        "launches": w,
        "hbm_bytes_per_launch": sum((r["hbm_read"] + r["hbm_write"]) * r["count"] for r in conv) / w,
        "algorithmic_bytes_per_launch": sum(r["bytes"] * r["count"] for r in conv) / w,
        "mfma_busy_count_weighted": sum(r["mfma_busy"] * r["count"] for r in conv) / w,
        "per_op": rows,
    }
    fam["ratio_to_algorithmic"] = fam["hbm_bytes_per_launch"] / fam["algorithmic_bytes_per_launch"]
    print(f"\nconv family: {fam['hbm_bytes_per_launch'] / 1e6:.1f} MB/launch by PMC vs "
          f"{fam['algorithmic_bytes_per_launch'] / 1e6:.1f} MB algorithmic (x{fam['ratio_to_algorithmic']:.2f}); "
          f"MFMA busy {fam['mfma_busy_count_weighted']:.3f} (count-weighted)")
    if json_out:
        with open(json_out, "w") as f:
            json.dump(fam, f, indent=1, default=float)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        args = sys.argv[2:]
        js = None
        if "--json" in args:
            i = args.index("--json")
            js = args[i + 1]
            args = args[:i] + args[i + 2:]
        report(args, js)
