"""Gradient error at every ResNet block output of both views (HIP fp32 vs fp64 oracle)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import spec  # noqa: E402
from greedy_multimodal_learning_amd.losses import blend_loss  # noqa: E402
from greedy_multimodal_learning_amd.model import MMTM_MVCNN  # noqa: E402
from oracle import gating_ref, model_ref, weights  # noqa: E402


def err(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max()) / (float(b.abs().max()) + 1e-30)


def instrument(model, store):
    for v in (0, 1):
        net = getattr(model, f"net_view_{v}")
        for li in range(1, 5):
            for bi, blk in enumerate(getattr(net, f"layer{li}")):
                name = f"v{v}.layer{li}.{bi}"
                orig = blk.forward

                def fwd(x, orig=orig, name=name):
                    y = orig(x)
                    y.retain_grad()
                    store[name] = y
                    return y
                blk.forward = fwd


train, _, _ = spec.trace_loaders(spec.TRACE_GPU)
_, x, y = train[0]
x, y = torch.from_numpy(x), torch.from_numpy(y)
m = weights.apply_to_module(MMTM_MVCNN(), seed=spec.SEED_MODEL).cuda()
o64 = weights.apply_to_module(model_ref.MMTM_MVCNN_Ref(), seed=spec.SEED_MODEL).double()
sh, s64 = {}, {}
instrument(m, sh)
instrument(o64, s64)
_, outs, _, _ = m(x.cuda())
blend_loss(outs, y.cuda()).backward()
_, oo, _, _ = o64(x.double())
gating_ref.blend_loss(oo, y).backward()
for k in sh:
    print(f"{k:16s} fwd {err(sh[k], s64[k]):.2e} grad {err(sh[k].grad, s64[k].grad):.2e}")
