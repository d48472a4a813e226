"""Run the bench's fused norms+SGD pass (k_group_sumsq<SGD>) a few times on the C2
model, for PMC collection (tools/gpu.sh pmcg:fetch / pmcg:write)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    dev = torch.device("cuda:0")
    from greedy_multimodal_learning_amd.engine import BalancedStep
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    torch.manual_seed(0)
    m = MMTM_MVCNN().to(dev)
    st = BalancedStep(m, lr=0.1)
    x = torch.randn(4, 2, 3, 64, 64, device=dev)
    y = torch.randint(0, 40, (4,), device=dev)
    st(x, y)
    torch.cuda.synchronize()
    for _ in range(10):
        st.norms.sums(grad_scale=1.0, lr=st.lr)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
