"""BN kernels alone (no autograd): fwd-train and bwd per trunk shape, for rocprof."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from greedy_multimodal_learning_amd import bn  # noqa: E402

CL = torch.channels_last
SHAPES = [(64, 64, 112, 112), (64, 64, 56, 56), (64, 128, 28, 28), (64, 256, 14, 14), (64, 512, 7, 7)]


def main():
    dev = torch.device("cuda:0")
    for (N, C, H, W) in SHAPES:
        x = torch.randn(N, C, H, W, device=dev).bfloat16().contiguous(memory_format=CL)
        dy = torch.randn_like(x)
        w = torch.ones(C, device=dev)
        b = torch.zeros(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
        for _ in range(20):
            y, sm, si = bn.bn_fwd_train(x, w, b, rm, rv, None, 0.1, 1e-5, True, None)
            bn.bn_bwd(dy, y, x, w, sm, si, True, False, dg, db, False)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(20_000_000)
        e0.record()
        for _ in range(20):
            y, sm, si = bn.bn_fwd_train(x, w, b, rm, rv, None, 0.1, 1e-5, True, None)
            bn.bn_bwd(dy, y, x, w, sm, si, True, False, dg, db, False)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 20 * 1e3
        mb = N * C * H * W * 2 / 1e6
        print(f"N{N} C{C} {H}x{W}: {mb:.1f} MB/tensor, fwd+bwd {t:.1f} us "
              f"(ideal@5TB/s ~{(mb * 10) / 5e3 * 1e3:.1f} us)", flush=True)


if __name__ == "__main__":
    main()
