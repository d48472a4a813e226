"""GPU trunk gradient error vs an fp64 CPU oracle, under the current MIOpen env."""
import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests", "golden"))
import numpy as np, torch
import spec
from oracle import weights, model_ref, gating_ref
from greedy_multimodal_learning_amd.model import MMTM_MVCNN
from greedy_multimodal_learning_amd.losses import blend_loss
fix = np.load(os.path.join(R, "tests/golden/golden_model.npz"))
dev = torch.device("cuda:0")
for cid in sys.argv[1:]:
    case = [c for c in spec.MODEL_CASES if c["id"] == cid][0]
    x, y = spec.model_inputs(case)
    o = weights.apply_to_module(model_ref.MMTM_MVCNN_Ref(), seed=0).double()
    _, outs, _, _ = o(torch.from_numpy(x).double(), curation_mode=case.get("cur", False), caring_modality=case.get("caring"))
    gating_ref.blend_loss(outs, torch.from_numpy(y)).backward()
    gn64 = np.array([float((q.grad**2).sum()) if q.grad is not None else 0 for _, q in o.named_parameters()])
    m = weights.apply_to_module(MMTM_MVCNN(), seed=0).to(dev)
    _, outs, _, _ = m(torch.from_numpy(x).to(dev), curation_mode=case.get("cur", False), caring_modality=case.get("caring"))
    blend_loss(outs, torch.from_numpy(y).to(dev)).backward()
    gn = np.array([float((q.grad.double()**2).sum()) if q.grad is not None else 0 for _, q in m.named_parameters()])
    live = gn64 > 0
    eg = np.abs(gn - gn64)[live] / gn64[live]
    er = np.abs(fix[cid + "/gn"] - gn64)[live] / gn64[live]
    print(f"{cid:7s} env={os.environ.get('DIAG_TAG','default'):12s} gpu rms={np.sqrt((eg**2).mean()):.2e} max={eg.max():.2e} | ref32 rms={np.sqrt((er**2).mean()):.2e} max={er.max():.2e}", flush=True)
