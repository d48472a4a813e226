"""Determinism / race screen of a weight-gradient launch (the layer-1 shape by default):
the same grouped launch repeated N times, alone and beside a busy kernel on another stream,
every output compared bitwise with the first and checked finite."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    mode = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    # neighbour: "conc" = the busy kernel runs beside the launch; "before" = it runs and
    # finishes first (only its leftover LDS contents remain)
    nb = sys.argv[3] if len(sys.argv) > 3 else "conc"
    from greedy_multimodal_learning_amd import build
    build.build()
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import conv as CV
    lib = L.load()
    L.check(lib.gm_conv_set_wgrad_loop(mode), "loop")
    dev = torch.device("cuda:0")
    N, H, W, C, K, G = 64, 56, 56, 64, 64, 2
    torch.manual_seed(0)
    x = torch.randn(G * N, H, W, C, device=dev).bfloat16()
    dy = torch.randn(G * N, H, W, K, device=dev).bfloat16()
    d = CV._desc_hw(N, H, W, C, K, 3, 3, 1, 1, 1, 1)
    need = lib.gm_conv2d_wgrad_grouped_scratch(ctypes.byref(d), G)
    scr = torch.empty(need, device=dev, dtype=torch.uint8)
    side = torch.cuda.Stream()
    big = torch.randn(8192, 8192, device=dev)

    def run(dw):
        L.check(lib.gm_conv2d_wgrad_grouped_bf16(ctypes.byref(d), G, dy.data_ptr(), x.data_ptr(), dw.data_ptr(),
                                                 K * 9 * C, C, 0, scr.data_ptr(), need, L.stream_of(dev)), "wgrad")
    ref = torch.empty(G, K, 3, 3, C, device=dev)
    run(ref)
    torch.cuda.synchronize()
    assert torch.isfinite(ref).all()
    bad = nonfinite = 0
    for i in range(reps):
        dw = torch.empty_like(ref)
        if i % 2:
            with torch.cuda.stream(side):
                big @ big  # a busy neighbour on another stream
            if nb == "before":
                side.synchronize()
        run(dw)
        torch.cuda.synchronize()
        if not torch.equal(dw, ref):
            bad += 1
            nonfinite += int(not torch.isfinite(dw).all())
            diff = (dw - ref).abs()
            print(f"rep {i}: {int((dw != ref).sum())} elements differ, max {float(diff[torch.isfinite(diff)].max()):.3e}, "
                  f"nonfinite {int((~torch.isfinite(dw)).sum())}", flush=True)
            if bad <= 3:  # where: (group, k, tap, c) of the differing elements
                idx = (dw != ref).nonzero()
                for dim, name in enumerate("gkrsc"):
                    print(f"   {name}: {sorted(set(idx[:, dim].tolist()))[:40]}", flush=True)
    print(f"mode {mode} neighbour {nb}: {reps} reps, {bad} differing, {nonfinite} with non-finite values", flush=True)


if __name__ == "__main__":
    main()
