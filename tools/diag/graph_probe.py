"""Probe which piece of the training step breaks hipGraph capture (run each
piece in its own process: python graph_probe.py <piece>)."""
import faulthandler
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
faulthandler.enable()
CL = torch.channels_last


def capture(fn, warm=1):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    g.replay()
    torch.cuda.synchronize()
    return out


def main(piece):
    dev = torch.device("cuda:0")
    from greedy_multimodal_learning_amd import conv, bn, pool
    if piece == "conv":
        m = conv.GMConv2d(64, 64, 3, padding=1, bias=False).to(dev).to(memory_format=CL)
        x = torch.randn(4, 64, 16, 16, device=dev).bfloat16().contiguous(memory_format=CL)
        capture(lambda: m(x))
    elif piece == "conv_bwd":
        m = conv.GMConv2d(64, 64, 3, padding=1, bias=False).to(dev).to(memory_format=CL)
        x = torch.randn(4, 64, 16, 16, device=dev).bfloat16().contiguous(memory_format=CL).requires_grad_(True)

        def f():
            y = m(x)
            y.float().sum().backward()
        capture(f)
    elif piece == "bn":
        m = bn.GMBatchNorm2d(64).to(dev)
        x = torch.randn(4, 64, 16, 16, device=dev).bfloat16().contiguous(memory_format=CL).requires_grad_(True)

        def f():
            y = m(x, relu=True)
            y.float().sum().backward()
        capture(f)
    elif piece == "pool":
        m = pool.GMMaxPool2d(3, 2, 1)
        x = torch.randn(4, 64, 16, 16, device=dev).bfloat16().contiguous(memory_format=CL).requires_grad_(True)

        def f():
            m(x).float().sum().backward()
        capture(f)
    elif piece == "mmtm":
        from greedy_multimodal_learning_amd.balanced_mmtm import MMTM_mitigate
        m = MMTM_mitigate(128, 128, 4).to(dev)
        a = torch.randn(4, 128, 8, 8, device=dev).bfloat16().contiguous(memory_format=CL).requires_grad_(True)
        b = torch.randn(4, 128, 8, 8, device=dev).bfloat16().contiguous(memory_format=CL).requires_grad_(True)

        def f():
            ya, yb, _, _ = m(a, b)
            (ya.float().sum() + yb.float().sum()).backward()
        capture(f)
    elif piece in ("model_fwd", "model_step", "norms"):
        from greedy_multimodal_learning_amd.engine import BalancedStep
        from greedy_multimodal_learning_amd.model import MMTM_MVCNN
        model = MMTM_MVCNN().to(dev)
        st = BalancedStep(model, lr=0.01)
        x = torch.randn(4, 2, 3, 64, 64, device=dev)
        y = torch.randint(0, 40, (4,), device=dev)
        st(x, y)
        if piece == "model_fwd":
            def f():
                with torch.no_grad():
                    return st.forward(x)
        elif piece == "norms":
            def f():
                return st.norms.sums(1.0, 0.01)
        else:
            def f():
                return st._fwd_bwd(x, y)
        capture(f)
    print("OK", piece, flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
