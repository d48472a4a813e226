"""Where the C5 step's PyTorch zero fills come from: one eager C5 engine step with
torch.zeros / zeros_like / Tensor.zero_ / Tensor.fill_ wrapped to count their (file:line)
call sites inside the package.

    python tools/diag/zero_fills.py [--workload C5] [--batch 32]
"""
import argparse
import collections
import sys
import traceback

import torch

sys.path.insert(0, ".")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="C5")
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    from greedy_multimodal_learning_amd.engine import BalancedStep
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN, MMTM_MVCNN_N
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    if a.workload == "C2":
        model, V = MMTM_MVCNN().to(dev), 2
        bn, mn = ["net_view_0", "net_view_1"], ["visual", "skeleton"]
    else:
        V, trunk = (4, "resnet18") if a.workload == "C4" else (12, "resnet50")
        model = MMTM_MVCNN_N(num_views=V, trunk=trunk).to(dev)
        bn, mn = model.branch_names(), model.mmtm_names()
    gate = Bias_Mitigation_Strong(epsilon=0.01, curation_windowsize=5, branchnames=bn, starting_epoch=1,
                                  MMTMnames=mn)
    step = BalancedStep(model, lr=0.1, gate=gate, compute_dtype=torch.bfloat16, channels_last=True, graphs=False,
                        branchnames=bn, MMTMnames=mn)
    step.on_epoch_begin(1)
    x = torch.randn(V, a.batch, 224, 224, 3, device=dev).bfloat16().permute(1, 0, 4, 2, 3)
    y = torch.randint(0, 40, (a.batch,), device=dev)
    for _ in range(2):
        step(x, y)
    torch.cuda.synchronize()
    sites = collections.Counter()

    def site():
        for fr in reversed(traceback.extract_stack()[:-2]):
            if "greedy_multimodal_learning_amd" in fr.filename:
                return f"{fr.filename.split('greedy_multimodal_learning_amd/')[-1]}:{fr.lineno} {fr.line}"
        return "?"

    z, zl, tz, tf = torch.zeros, torch.zeros_like, torch.Tensor.zero_, torch.Tensor.fill_

    def wz(*args, **kw):
        sites["zeros " + site()] += 1
        return z(*args, **kw)

    def wzl(*args, **kw):
        sites["zeros_like " + site()] += 1
        return zl(*args, **kw)

    def wtz(self):
        sites["zero_ " + site()] += 1
        return tz(self)

    def wtf(self, v):
        sites["fill_ " + site()] += 1
        return tf(self, v)

    torch.zeros, torch.zeros_like, torch.Tensor.zero_, torch.Tensor.fill_ = wz, wzl, wtz, wtf
    try:
        step(x, y)
        torch.cuda.synchronize()
    finally:
        torch.zeros, torch.zeros_like, torch.Tensor.zero_, torch.Tensor.fill_ = z, zl, tz, tf
    for k, v in sites.most_common(30):
        print(f"{v:4d}  {k}")


if __name__ == "__main__":
    main()
