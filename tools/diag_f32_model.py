"""Per-parameter gradient error of the fp32 HIP MMTM_MVCNN and of the fp32 CPU oracle,
both against the float64 oracle, on the first batch of the GPU trace (diagnostic)."""
import os
import sys

import numpy as np
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


train, _, _ = spec.trace_loaders(spec.TRACE_GPU)
_, x, y = train[0]
x, y = torch.from_numpy(x), torch.from_numpy(y)
m = weights.apply_to_module(MMTM_MVCNN(), seed=spec.SEED_MODEL).cuda()
o32 = weights.apply_to_module(model_ref.MMTM_MVCNN_Ref(), seed=spec.SEED_MODEL)
o64 = weights.apply_to_module(model_ref.MMTM_MVCNN_Ref(), seed=spec.SEED_MODEL).double()
_, outs, _, _ = m(x.cuda())
blend_loss(outs, y.cuda()).backward()
for o, dt in ((o32, torch.float32), (o64, torch.float64)):
    _, oo, _, _ = o(x.to(dt))
    gating_ref.blend_loss(oo, y).backward()
p32, p64 = dict(o32.named_parameters()), dict(o64.named_parameters())
rows = []
for n, p in m.named_parameters():
    if p.grad is None:
        continue
    rows.append((err(p.grad, p64[n].grad), err(p32[n].grad, p64[n].grad), n))
e_h = np.array([r[0] for r in rows])
e_c = np.array([r[1] for r in rows])
print(f"rms hip {np.sqrt((e_h ** 2).mean()):.3e} cpu32 {np.sqrt((e_c ** 2).mean()):.3e}; "
      f"median hip {np.median(e_h):.3e} cpu32 {np.median(e_c):.3e}")
for e, e32, n in sorted(rows, key=lambda r: -r[0] / (r[1] + 1e-12))[:25]:
    print(f"{n:50s} hip {e:.3e}  cpu32 {e32:.3e}")

# ---- MMTM site alone: fp32 NCHW / NHWC on the GPU vs the oracle in float64 ----
from greedy_multimodal_learning_amd.balanced_mmtm import MMTM_mitigate  # noqa: E402
from oracle.mmtm_ref import MMTMRef as MMTM_Ref  # noqa: E402
for C, H in ((128, 16), (256, 8), (512, 4)):
    g = torch.Generator().manual_seed(C)
    xv, xs = torch.randn(8, C, H, H, generator=g), torch.randn(8, C, H, H, generator=g)
    dyv, dys = torch.randn(8, C, H, H, generator=g), torch.randn(8, C, H, H, generator=g)
    ref = MMTM_Ref(C, C, 4).double()
    mm = MMTM_mitigate(C, C, 4, device="cuda:0").cuda()
    mm.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    rv, rs = xv.double().requires_grad_(True), xs.double().requires_grad_(True)
    ov, os_, _, _ = ref(rv, rs)
    (ov * dyv.double()).sum().add_((os_ * dys.double()).sum()).backward()
    for lay in (torch.contiguous_format, torch.channels_last):
        gv = xv.cuda().contiguous(memory_format=lay).requires_grad_(True)
        gs = xs.cuda().contiguous(memory_format=lay).requires_grad_(True)
        yv, ys, _, _ = mm(gv, gs)
        (yv * dyv.cuda()).sum().add_((ys * dys.cuda()).sum()).backward()
        print(C, "NHWC" if lay == torch.channels_last else "NCHW", "y", err(yv, ov), err(ys, os_),
              "dx", err(gv.grad, rv.grad), err(gs.grad, rs.grad))
