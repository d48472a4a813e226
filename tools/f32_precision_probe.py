"""Where does the fp32 drop-in's gradient error come from?  (test_gpu_model.py m224 cases:
per-parameter gradient norms of view 0's BatchNorms ~1e-3 off the fp64 oracle where the
reference's own fp32 run is ~1e-6 off.)

Runs the m224 case (B=1, 224x224, seed 4) fwd + bwd on the HIP fp32 path under a few
configurations and prints, per configuration, the gradient-norm error against the
oracle in float64 and the worst parameters:
  streams   the default (view 1 on a side stream)
  nostream  GM_VIEW_STREAMS=0 (both trunks on one stream)
  twice     the default run again (run-to-run determinism)

    python tools/f32_precision_probe.py [--case m224]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import spec
    from oracle import gating_ref, model_ref, weights
    from greedy_multimodal_learning_amd.losses import blend_loss
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="m224")
    ap.add_argument("--blocks", action="store_true", help="per-block forward/gradient error (first divergence)")
    a = ap.parse_args()
    case = [c for c in spec.MODEL_CASES if c["id"] == a.case][0]
    dev = torch.device("cuda:0")
    x, y = spec.model_inputs(case)
    X, Y = torch.from_numpy(x), torch.from_numpy(y)
    o = weights.apply_to_module(model_ref.MMTM_MVCNN_Ref(), seed=spec.SEED_MODEL).double()
    _, outs, _, _ = o(X.double())
    gating_ref.blend_loss(outs, Y).backward()
    g64 = {n: p.grad.double() for n, p in o.named_parameters()}

    def run(streams):
        os.environ["GM_VIEW_STREAMS"] = "1" if streams else "0"
        m = weights.apply_to_module(MMTM_MVCNN(), seed=spec.SEED_MODEL).to(dev)
        m.train(True)
        _, outs, _, _ = m(X.to(dev))
        blend_loss(outs, Y.to(dev)).backward()
        torch.cuda.synchronize()
        return {n: p.grad.detach().double().cpu() for n, p in m.named_parameters()}

    if a.blocks:
        return blocks(o, X, Y, dev, g64)
    res = {"streams": run(True), "nostream": run(False), "twice": run(True)}
    names = list(g64)
    for k, g in res.items():
        e = np.array([float(((g[n] - g64[n]).norm() / (g64[n].norm() + 1e-300))) for n in names])
        worst = np.argsort(-e)[:5]
        print(f"{k:9s} grad rel-L2 err vs fp64: max {e.max():.2e} median {np.median(e):.2e}  worst: " +
              ", ".join(f"{names[i]} {e[i]:.1e}" for i in worst))
    d = max(float((res["streams"][n] - res["twice"][n]).abs().max()) for n in names)
    d2 = max(float((res["streams"][n] - res["nostream"][n]).abs().max()) for n in names)
    print(f"max |streams - twice| = {d:.3e}; max |streams - nostream| = {d2:.3e}")


def blocks(o, X, Y, dev, g64):
    """Forward outputs and their gradients at every ResNet block / MMTM site of both models
    (hooks on the same module names), relative L2 error of the HIP fp32 run vs float64, in
    execution order: the first row where the error jumps is the op that loses precision."""
    import spec
    from oracle import gating_ref, weights
    from greedy_multimodal_learning_amd.losses import blend_loss
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    m = weights.apply_to_module(MMTM_MVCNN(), seed=spec.SEED_MODEL).to(dev)
    m.train(True)
    watch = []
    for v in (0, 1):
        watch += [f"net_view_{v}.conv1"] + [f"net_view_{v}.layer{l}.{j}" for l in (1, 2, 3, 4) for j in (0, 1)]
    watch += ["mmtm2", "mmtm3", "mmtm4"]
    for v in (0, 1):  # inside the strided block of layer 4: conv outputs = BatchNorm inputs
        watch += [f"net_view_{v}.layer4.0.{c}" for c in ("conv1", "conv2", "downsample.0")]

    def hook(store):
        def fn(mod, inp, out):
            outs = out if isinstance(out, tuple) else (out,)
            ts = [t for t in outs[:2] if torch.is_tensor(t)]
            for t in ts:
                if t.requires_grad:
                    t.retain_grad()
            store.append(ts)
        return fn
    rec = {}
    for mm, tag in ((m, "hip"), (o, "ref")):
        mods = dict(mm.named_modules())
        for n in watch:
            rec[(tag, n)] = []
            mods[n].register_forward_hook(hook(rec[(tag, n)]))
    o.zero_grad(set_to_none=True)
    _, outs, _, _ = o(X.double())
    gating_ref.blend_loss(outs, Y).backward()
    _, outs, _, _ = m(X.to(dev))
    blend_loss(outs, Y.to(dev)).backward()
    torch.cuda.synchronize()

    def rel(a, b):
        a, b = a.detach().double().cpu(), b.detach().double().cpu()
        return float((a - b).norm() / (b.norm() + 1e-300))
    for n in watch:
        hs, rs = rec[("hip", n)][0], rec[("ref", n)][0]
        for k, (h, r) in enumerate(zip(hs, rs)):
            gh = h.grad if h.grad is not None else None
            gr = r.grad if r.grad is not None else None
            ge = rel(gh, gr) if (gh is not None and gr is not None) else float("nan")
            flips = int(((h.detach().double().cpu() > 0) != (r.detach().double().cpu() > 0)).sum())
            print(f"{n:28s}[{k}] fwd {rel(h, r):.2e}  grad {ge:.2e}  sign flips vs fp64 {flips}")


if __name__ == "__main__":
    main()
