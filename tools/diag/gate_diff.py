"""Host gate vs on-device gate, step by step: first step and parameters that differ."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def make(device_gate, dev):
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    from greedy_multimodal_learning_amd.engine import BalancedStep
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    torch.manual_seed(0)
    m = MMTM_MVCNN().to(dev)
    gate = Bias_Mitigation_Strong(epsilon=2e-3, curation_windowsize=2, branchnames=["net_view_0", "net_view_1"],
                                  starting_epoch=1)
    st = BalancedStep(m, lr=0.05, gate=gate, graphs=False, device_gate=device_gate)
    st.on_epoch_begin(1)
    return m, st, gate


def main():
    dev = torch.device("cuda:0")
    mh, sh, gh = make(False, dev)
    md, sd, gd = make(True, dev)
    g = torch.Generator(device=dev).manual_seed(5)
    xs = [torch.randn(4, 2, 3, 64, 64, device=dev, generator=g) for _ in range(3)]
    ys = [torch.randint(0, 40, (4,), device=dev, generator=g) for _ in range(3)]
    for i in range(6):
        fh = (sh.flags.curation_mode, sh.flags.caring_modality)
        sd.sync_gate()
        fd = (sd.flags.curation_mode, sd.flags.caring_modality)
        lh = float(sh(xs[i % 3], ys[i % 3]))
        ld = float(sd(xs[i % 3], ys[i % 3]))
        sd.sync_gate()
        a, b = mh.state_dict(), md.state_dict()
        bad = [(k, float((a[k].float() - b[k].float()).abs().max())) for k in a
               if not torch.equal(a[k], b[k])]
        bad.sort(key=lambda t: -t[1])
        print(f"step {i}: flags in h{fh} d{fd}  loss h {lh:.6f} d {ld:.6f}  dBDR h {gh.d_BDR:.6f} d {gd.d_BDR:.6f}  "
              f"differing tensors {len(bad)}: {bad[:5]}", flush=True)


if __name__ == "__main__":
    main()
