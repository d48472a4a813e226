"""How a captured two-branch hipGraph is executed: two chains of N spin kernels
(torch.cuda._sleep, ~T us each) forked from one root and joined at the end, captured
with the branches issued one after the other ("seq") or alternately ("inter").  Wall
time per replay ~N*T means the branches overlap, ~2N*T that they serialise; with
"seqlag" the second-issued branch's chain is shorter, to see whether it waits for the
first branch's queue tail.

    python tools/diag/graph_fork_probe.py [N] [cycles]
"""
import sys
import time

import torch


BIG = {}


def work(cyc):
    """spin kernel (one workgroup), or with BIG set a whole-GPU elementwise pass"""
    if BIG:
        BIG["t"].mul_(1.0001)
    else:
        torch.cuda._sleep(cyc)


def build(order, n, cyc, main, side):
    g = torch.cuda.CUDAGraph()
    x = torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        x.add_(1)
        side.wait_stream(torch.cuda.current_stream())
        if order == "seq":
            with torch.cuda.stream(side):
                for _ in range(n):
                    work(cyc)
            for _ in range(n):
                work(cyc)
        elif order == "seqrev":
            for _ in range(n):
                work(cyc)
            with torch.cuda.stream(side):
                for _ in range(n):
                    work(cyc)
        else:
            for _ in range(n):
                with torch.cuda.stream(side):
                    work(cyc)
                work(cyc)
        torch.cuda.current_stream().wait_stream(side)
        x.add_(1)
    return g


def build_segments(segs, n, cyc, side):
    """segs fork/join segments of two n-kernel branches, like the step's MMTM sites"""
    g = torch.cuda.CUDAGraph()
    x = torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(segs):
            x.add_(1)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(n):
                    work(cyc)
            for _ in range(n):
                work(cyc)
            torch.cuda.current_stream().wait_stream(side)
        x.add_(1)
    return g


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    cyc = int(sys.argv[2]) if len(sys.argv) > 2 else 40000
    if "--big" in sys.argv:
        BIG["t"] = torch.ones(32 << 20, device="cuda")  # 128 MB: ~40 us per pass
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    one = timeit(lambda: work(cyc), 50)
    print(f"one spin kernel: {one:.1f} us (eager, incl. launch)")
    for order in ("seq", "seqrev", "inter"):
        g = build(order, n, cyc, main_s, side)
        t = timeit(g.replay)
        print(f"{order:7s} n={n}: {t:8.1f} us per replay = {t / (n * one):.2f} x one chain", flush=True)
    g = build_segments(8, n, cyc, side)
    t = timeit(g.replay)
    print(f"8 segments n={n}: {t:8.1f} us per replay = {t / (8 * n * one):.2f} x one chain per segment", flush=True)


if __name__ == "__main__":
    main()
