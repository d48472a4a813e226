"""Diagnostic: stacked (vtrunk) vs per-view bf16 gradients, directly, for one model kind,
with the epilogue BatchNorm statistics on and off, and a repeat of each (determinism)."""
import sys

import torch

sys.path.insert(0, ".")
from greedy_multimodal_learning_amd import vtrunk  # noqa: E402
from greedy_multimodal_learning_amd.losses import blend_loss  # noqa: E402
from greedy_multimodal_learning_amd.model import MMTM_MVCNN, MMTM_MVCNN_N  # noqa: E402

CL = torch.channels_last
kind = sys.argv[1] if len(sys.argv) > 1 else "n4-r18"
dev = torch.device("cuda:0")
torch.manual_seed(11)
B, H = 8, 64
if kind == "mvcnn2":
    V, make = 2, MMTM_MVCNN
else:
    V = int(kind[1])
    make = lambda: MMTM_MVCNN_N(num_views=V, trunk="resnet50" if kind.endswith("r50") else "resnet18")  # noqa
ms = [make().to(dev).to(memory_format=CL).train() for _ in range(5)]
for m in ms[1:]:
    m.load_state_dict(ms[0].state_dict())
x = torch.randn(B, V, 3, H, H, device=dev).bfloat16()
y = torch.randint(0, 40, (B,), device=dev)
runs = [("stacked-epi", True, True), ("per-view", False, True), ("stacked-noepi", True, False),
        ("stacked-noepi-2", True, False), ("stacked-epi-2", True, True)]
grads = {}
for m, (name, on, epi) in zip(ms, runs):
    vtrunk.ENABLED, vtrunk.EPI_BN_STATS = on, epi
    with torch.autocast("cuda", dtype=torch.bfloat16):
        _, o, _, _ = m(x)
    blend_loss([t.float() for t in o], y).backward()
    grads[name] = torch.cat([p.grad.double().flatten() for p in m.parameters()])
vtrunk.ENABLED, vtrunk.EPI_BN_STATS = True, True
ref = grads["per-view"]
for k, g in grads.items():
    print(f"{kind} {k:16s} vs per-view {float((g - ref).norm() / ref.norm()):.3e}   "
          f"vs stacked-noepi {float((g - grads['stacked-noepi']).norm() / ref.norm()):.3e}", flush=True)
