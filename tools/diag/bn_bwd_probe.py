"""Isolated timing of the ReLU-after-BN backward forms on the trunk's view-grouped shapes:
the single-launch k_bn_bwd_fused<BWD_RELUX> (gm_bn_bwd_grouped_bf16) against the finalize +
streaming apply that follows statistics from the input-gradient epilogue
(gm_bn_bwd_stats_finalize_grouped + gm_bn_bwd_apply_grouped_bf16).

    python tools/diag/bn_bwd_probe.py
"""
import sys

import torch

sys.path.insert(0, ".")
from greedy_multimodal_learning_amd import vtrunk  # noqa: E402

CL = torch.channels_last


def timeit(fn, n=20, reps=5):
    """Device time per call: n calls captured in one HIP graph, replayed (no host overhead)."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (n * reps) * 1e3


def main():
    dev = torch.device("cuda:0")
    G = 2
    for N, C, H in ((64, 64, 56), (64, 128, 28), (64, 256, 14), (64, 512, 7)):
        xb = torch.randn(G * N, C, H, H, device=dev).bfloat16().contiguous(memory_format=CL)
        dz = torch.randn_like(xb).contiguous(memory_format=CL)
        gam = [torch.rand(C, device=dev) + 0.5 for _ in range(G)]
        bet = [torch.zeros(C, device=dev) for _ in range(G)]
        sm = torch.zeros(G, C, device=dev)
        si = torch.ones(G, C, device=dev)
        coef = torch.cat([torch.ones(G, C, device=dev), torch.zeros(G, C, device=dev)], 1).contiguous()
        M = N * H * H
        rows = 256  # k_conv_rw's partial rows per group (the h9 / ring epilogues write more)
        part = torch.zeros(G * 2 * C * (rows + 1) + G * 4 * C, device=dev)
        t_fused = timeit(lambda: vtrunk._bn_backward(dz, None, xb, G, gam, bet, sm, si, True, False, coef, True, True))
        t_split = timeit(lambda: vtrunk._bn_backward_from_stats(dz, xb, G, gam, bet, sm, si, coef, part, rows,
                                                                True, True))
        mb = 3 * xb.numel() * 2 / 1e6
        print(f"N={N} C={C} H={H}: single-launch {t_fused:7.1f} us | finalize+apply {t_split:7.1f} us "
              f"(apply {mb:.0f} MB -> {mb / t_split:.2f} TB/s incl. finalize)", flush=True)


if __name__ == "__main__":
    main()
