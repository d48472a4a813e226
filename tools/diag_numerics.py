"""Diagnose where GPU-vs-reference numeric drift comes from (trunk vs MMTM)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
import numpy as np, torch
import spec
from oracle import weights, mmtm_ref
from greedy_multimodal_learning_amd.model import MMTM_MVCNN
from greedy_multimodal_learning_amd.losses import blend_loss

fix = np.load("tests/golden/golden_model.npz")
dev = torch.device("cuda:0")

def run(case, use_ref_mmtm, tf32, cudnn):
    torch.backends.cudnn.allow_tf32 = tf32
    torch.backends.cuda.matmul.allow_tf32 = tf32
    torch.backends.cudnn.enabled = cudnn
    m = MMTM_MVCNN()
    if use_ref_mmtm:
        for i, C in ((2, 128), (3, 256), (4, 512)):
            setattr(m, f"mmtm{i}", mmtm_ref.MMTMRef(C, C, 4))
    weights.apply_to_module(m, seed=spec.SEED_MODEL)
    m = m.to(dev)
    for i in (2, 3, 4):
        mm = getattr(m, f"mmtm{i}")
        mm.running_avg_weight_visual = mm.running_avg_weight_visual.to(dev)
        mm.running_avg_weight_skeleton = mm.running_avg_weight_skeleton.to(dev)
    m.train(True)
    x, y = spec.model_inputs(case)
    mean, outs, _, _ = m(torch.from_numpy(x).to(dev), curation_mode=case.get("cur", False), caring_modality=case.get("caring"))
    loss = blend_loss(outs, torch.from_numpy(y).to(dev))
    loss.backward()
    p = case["id"] + "/"
    lg = mean.detach().cpu().numpy()
    e_lg = np.abs(lg - fix[p + "logits"]).max() / np.abs(fix[p + "logits"]).max()
    gn = np.array([float((q.grad.double() ** 2).sum()) if q.grad is not None else 0.0 for _, q in m.named_parameters()])
    rel = np.abs(gn - fix[p + "gn"]) / np.maximum(np.abs(fix[p + "gn"]), 1e-30)
    return e_lg, rel.max(), np.median(rel)

for case in spec.MODEL_CASES:
    for ref_mmtm in (False, True):
        for tf32, cudnn in ((True, True), (False, True), (False, False)):
            e = run(case, ref_mmtm, tf32, cudnn)
            print(f"{case['id']:6s} ref_mmtm={ref_mmtm!s:5s} tf32={tf32!s:5s} miopen={cudnn!s:5s}  logits_rel={e[0]:.2e}  gn_rel max={e[1]:.2e} med={e[2]:.2e}", flush=True)
