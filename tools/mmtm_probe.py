"""HBM roofline of the MMTM squeeze (global-average-pool of both views' activations,
k_colreduce_nhwc via gm_mmtm_spatial_reduce) at the north-star batch 256 on the largest
site (s2: 128 channels x 28x28 per view, both views = 102.8 MB of bf16 per launch).

Launches rotate over `pairs` distinct activation pairs (default 4 = 411 MB > the 256 MiB
Infinity Cache), so every launch reads its bytes from HBM, not from a cache the
previous launch warmed (MI355X_MICROARCH.md, Infinity Cache residency rule).

    python tools/mmtm_probe.py run                  # the launches (under rocprofv3 --pmc)
    python tools/mmtm_probe.py report FETCH_DIR WRITE_DIR --json out.json
    (bench.py imports measure() for its `roofline_mmtm` object)
"""
import argparse
import csv
import glob
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
C, H = 128, 28
KERNEL = "k_colreduce_nhwc"


def make_pairs(dev, B, pairs):
    from greedy_multimodal_learning_amd import _lib as L  # noqa: F401
    CL = torch.channels_last
    g = torch.Generator(device=dev).manual_seed(3)
    out = []
    for _ in range(pairs):
        xv = torch.randn(B, C, H, H, device=dev, generator=g).bfloat16().contiguous(memory_format=CL)
        xs = torch.randn(B, C, H, H, device=dev, generator=g).bfloat16().contiguous(memory_format=CL)
        sq = torch.empty(B, 2 * C, device=dev)
        out.append([dict(x=xv, C=C, HW=H * H, out=sq, ld_out=2 * C, scale=1.0 / (H * H)),
                    dict(x=xs, C=C, HW=H * H, out=sq, out_off=C, ld_out=2 * C, scale=1.0 / (H * H))])
    return out


def measure(dev, B=256, pairs=4, reps=20):
    """(algorithmic bytes per launch, seconds per launch, bytes rotated over): HIP events
    on the launch stream behind a device sleep, launches cycling over the pairs."""
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import ops
    probs = make_pairs(dev, B, pairs)

    def op(i):
        ops.spatial_reduce(probs[i % pairs], B, L.GM_BF16, L.GM_NHWC, dev)
    for i in range(pairs):
        op(i)
    torch.cuda.synchronize()
    torch.cuda._sleep(20_000_000)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        op(i)
    e1.record()
    torch.cuda.synchronize()
    nbytes = 2 * B * C * H * H * 2
    return nbytes, e0.elapsed_time(e1) / reps / 1e3, nbytes * pairs


def _counter_means(d, counter):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
                    vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["run", "report", "ab"])
    ap.add_argument("dirs", nargs="*")
    ap.add_argument("--json", default=None)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    if a.mode == "ab":  # interleaved rounds of the unroll forms in one process
        from greedy_multimodal_learning_amd import _lib as L
        lib = L.load()
        res = {u: [] for u in ((256, 4), (-256, 4), (-256, 8), (-1024, 4))}
        for _ in range(5):
            for u in res:
                L.check(lib.gm_mmtm_set_reduce_form(*u), "set_reduce_form")
                nb, secs, _ = measure(torch.device("cuda:0"), a.batch)
                res[u].append(secs * 1e6)
        for u, ts in res.items():
            ts.sort()
            print(f"threads (negative: nontemporal), unroll {u}: median {ts[len(ts) // 2]:.2f} us  min {ts[0]:.2f} us  "
                  f"-> {nb / ts[len(ts) // 2] / 1e3:.0f} GB/s ({nb / ts[len(ts) // 2] / 1e3 / 8000:.3f} of 8 TB/s)")
        return
    if a.mode == "run":
        nb, secs, rot = measure(torch.device("cuda:0"), a.batch)
        print(f"{nb / 1e6:.1f} MB per launch, {secs * 1e6:.2f} us, {nb / secs / 1e9:.0f} GB/s "
              f"(rotating over {rot / 1e6:.0f} MB)")
        return
    fetch, nf = _counter_means(a.dirs[0], "FETCH_SIZE")
    write, nw = _counter_means(a.dirs[1], "WRITE_SIZE")
    alg = 2 * a.batch * C * H * H * 2 + a.batch * 2 * C * 4
    rd, wr = 2 * fetch * 1024, write * 1024
    out = {"kernel": f"gm::{KERNEL} (MMTM squeeze, site s2, B={a.batch}, both views)",
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over tools/mmtm_probe.py "
                     "run (launches rotating over 4 distinct activation pairs = 411 MB > 256 MiB Infinity Cache); "
                     "FETCH_SIZE doubled (gfx950 reports half of 16-B/lane streaming reads, MI355X_MICROARCH.md "
                     "HBM section); KB = 1024 B",
           "dispatches": [nf, nw], "fetch_size_kb": fetch, "write_size_kb": write,
           "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
           "algorithmic_bytes_per_launch": alg, "ratio_to_algorithmic": round((rd + wr) / alg, 4)}
    s = json.dumps(out, indent=1)
    print(s)
    if a.json:
        with open(a.json, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
