#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ by importing the REFERENCE.

Runs only in the build container (it needs /root/reference, read-only).  The
reference's missing dependencies are replaced by shims that carry no reference
code:

* `gin`, `gin.config`  - `configurable` is the identity decorator.
* `argh`               - unused stub.
* `torchvision.models` - `resnet18` = oracle.resnet_ref.resnet18 (torchvision
                         is not vendored upstream; names/init restated there).
* `torchvision.transforms` - inert stubs (only dataset.py touches them).
* `Tensor.to("cuda:*")` -> cpu while the reference builds MMTM_mitigate
  (`src/balanced_mmtm.py:30-31` hard-codes a CUDA device).
* `np.Inf`             - NumPy 2 removed it (`src/callbacks.py:403-413`).

Inputs are regenerated in the tests from the same seeds (tests/golden/spec.py),
so the .npz files hold mostly outputs.

Usage:  python tests/golden/make_golden.py [--ref /root/reference]
"""
import argparse
import os
import pickle
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from oracle import resnet_ref, weights  # noqa: E402
import spec  # noqa: E402


def install_shims(ref):
    def configurable(fn=None, *a, **k):
        if fn is None or not callable(fn):
            return lambda f: f
        return fn
    gin = types.ModuleType("gin")
    gin.configurable = configurable
    gin_config = types.ModuleType("gin.config")
    gin_config._CONFIG = {}
    gin_config._OPERATIVE_CONFIG = {}
    gin.config = gin_config
    gin.parse_config_files_and_bindings = lambda *a, **k: None
    sys.modules["gin"] = gin
    sys.modules["gin.config"] = gin_config
    argh = types.ModuleType("argh")
    argh.dispatch_command = lambda *a, **k: None
    sys.modules["argh"] = argh
    tv = types.ModuleType("torchvision")
    tvm = types.ModuleType("torchvision.models")
    tvm.resnet18 = resnet_ref.resnet18
    tvm.resnet50 = resnet_ref.resnet50
    tvt = types.ModuleType("torchvision.transforms")
    for n in ("Compose", "ToTensor", "Normalize", "ToPILImage", "RandomHorizontalFlip"):
        setattr(tvt, n, lambda *a, **k: (lambda x: x))
    tv.models, tv.transforms = tvm, tvt
    sys.modules.update({"torchvision": tv, "torchvision.models": tvm, "torchvision.transforms": tvt})
    np.Inf = np.inf
    os.environ.setdefault("DATA_DIR", tempfile.gettempdir())
    orig_to = torch.Tensor.to

    def to_cpu(self, *a, **k):
        if a and isinstance(a[0], str) and a[0].startswith("cuda"):
            a = ("cpu",) + a[1:]
        if a and isinstance(a[0], torch.device) and a[0].type == "cuda":
            a = (torch.device("cpu"),) + a[1:]
        return orig_to(self, *a, **k)
    torch.Tensor.to = to_cpu
    sys.path.insert(0, ref)


def tt(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def mmtm_cases(R):
    """F1: MMTM_mitigate unit cases, every mode, fwd + bwd + running average."""
    out = {}
    for case in spec.MMTM_CASES:
        cid, B, C, H, W = case["id"], case["B"], case["C"], case["H"], case["W"]
        kw = dict(SEonly=case.get("SEonly", False), shareweight=case.get("shareweight", False))
        m = R.MMTM_mitigate(C, C, 4, **kw)
        weights.apply_to_module(m, seed=spec.SEED_MMTM)
        xv, xs, dyv, dys = spec.mmtm_inputs(case)
        avg = spec.mmtm_avg(case)
        # k warm-up forwards advance the running averages / step counter first
        for k in range(case.get("warm", 0)):
            wv, ws = spec.mmtm_warm_inputs(case, k)
            with torch.no_grad():
                m(tt(wv), tt(ws))
        Xv = tt(xv).requires_grad_(True)
        Xs = tt(xs).requires_grad_(True)
        mode = case["mode"]
        kwargs = dict(return_scale=True, return_squeezed_mps=(mode == "normal"),
                      turnoff_cross_modal_flow=(mode == "turnoff"),
                      average_squeezemaps=[tt(avg[0]), tt(avg[1])] if mode == "turnoff" else None,
                      curation_mode=mode.startswith("cur"),
                      caring_modality=int(mode[-1]) if mode.startswith("cur") else 0)
        Yv, Ys, scales, sq = m(Xv, Xs, **kwargs)
        (Yv * tt(dyv)).sum().backward(retain_graph=True)
        (Ys * tt(dys)).sum().backward()
        p = f"{cid}/"
        out[p + "Yv"], out[p + "Ys"] = Yv.detach().numpy(), Ys.detach().numpy()
        out[p + "ev"], out[p + "es"] = scales[0].detach().numpy(), scales[1].detach().numpy()
        if sq is not None:
            out[p + "sqv"], out[p + "sqs"] = sq[0].detach().numpy(), sq[1].detach().numpy()
        out[p + "dXv"], out[p + "dXs"] = Xv.grad.numpy(), Xs.grad.numpy()
        for n, prm in m.named_parameters():
            out[p + "grad." + n] = (prm.grad.numpy() if prm.grad is not None
                                    else np.full(prm.shape, np.nan, np.float32))
        for k in [k for k in out if k.startswith(p)]:
            if out[k].size > spec.FULL_LIMIT:
                for suf, v in spec.signature(k, out.pop(k)).items():
                    out[k + suf] = v
        out[p + "ra_v"] = m.running_avg_weight_visual.numpy()
        out[p + "ra_s"] = m.running_avg_weight_skeleton.numpy()
        out[p + "step"] = np.array(m.step)
    return out


def model_cases(R):
    """F2: full MMTM_MVCNN forward/backward + per-group sums (compute_BDR inputs)."""
    from src import callbacks as C
    out = {}
    for case in spec.MODEL_CASES:
        cid = case["id"]
        model = R.MMTM_MVCNN(saving_mmtm_scales=True, saving_mmtm_squeeze_array=True)
        weights.apply_to_module(model, seed=spec.SEED_MODEL)
        model.train(True)
        x, y = spec.model_inputs(case)
        X = tt(x)
        out_mean, outs, scales, sqs = model(X, curation_mode=case.get("cur", False),
                                            caring_modality=case.get("caring", None))
        loss = spec_blend_loss(outs, tt(y))
        loss.backward()
        p = f"{cid}/"
        out[p + "logits"] = out_mean.detach().numpy()
        out[p + "logits0"] = outs[0].detach().numpy()
        out[p + "logits1"] = outs[1].detach().numpy()
        out[p + "loss"] = np.array(float(loss.detach()))
        for i, (sc, sq) in enumerate(zip(scales, sqs)):
            out[p + f"scale{i}_v"], out[p + f"scale{i}_s"] = sc[0].detach().numpy(), sc[1].detach().numpy()
            out[p + f"sq{i}_v"], out[p + f"sq{i}_s"] = sq[0].detach().numpy(), sq[1].detach().numpy()
        names, wn, gn = [], [], []
        for n, prm in model.named_parameters():
            names.append(n)
            g = prm.grad if prm.grad is not None else torch.zeros_like(prm)
            wn.append(float((prm ** 2).sum()))
            gn.append(float((g ** 2).sum()))
        out[p + "param_names"] = np.array(names)
        out[p + "wn"] = np.array(wn)
        out[p + "gn"] = np.array(gn)
        cb = C.Bias_Mitigation_Strong(epsilon=0.01, curation_windowsize=5,
                                      branchnames=["net_view_0", "net_view_1"])
        cb.set_model(model, ignore=False)
        cb.M_bypass_modal_0 = cb.M_bypass_modal_1 = cb.M_main_modal_0 = cb.M_main_modal_1 = 0
        if not case.get("cur", False):
            out[p + "d_BDR"] = np.array(cb.compute_BDR())
        # sampled gradient values of every parameter (positions from the spec rng)
        for n, prm in model.named_parameters():
            if prm.grad is not None:
                idx = spec.sample_idx(n, prm.numel())
                out[p + "gsample." + n] = prm.grad.reshape(-1)[idx].numpy()
        out[p + "bn_rm"] = model.net_view_0.layer2[0].bn1.running_mean.numpy()
        out[p + "bn_rv"] = model.net_view_1.layer4[1].bn2.running_var.numpy()
    return out


def spec_blend_loss(outs, y):
    import train as T  # reference train.py (blend_loss, acc)
    return T.blend_loss(outs, y)


def trace_case(R, case=None, ev=None, tag="trace"):
    """F3: the reference's own Model_.train_loop, guided gating, per-step trace."""
    from src import callbacks as C
    from src.framework import Model_
    import train as T
    case = spec.TRACE if case is None else case
    ev = spec.TRACE_EVAL if ev is None else ev
    model = R.MMTM_MVCNN()
    weights.apply_to_module(model, seed=spec.SEED_MODEL)
    train, valid, test = spec.trace_loaders(case)
    conv = lambda L: [(np.array(i), tt(x), tt(y)) for (i, x, y) in L]  # noqa: E731
    opt = torch.optim.SGD(model.parameters(), lr=case["lr"], momentum=0, weight_decay=0)
    gate = C.Bias_Mitigation_Strong(epsilon=case["epsilon"], curation_windowsize=case["window"],
                                    branchnames=["net_view_0", "net_view_1"],
                                    starting_epoch=case["starting_epoch"])
    rec = []

    class Rec(C.Callback):
        def on_batch_end(self, batch, logs):
            if "d_BDR" in logs:
                rec.append((logs["loss"], logs["d_BDR"], logs["curation_mode"],
                            -1 if logs["caring_modality"] is None else logs["caring_modality"],
                            logs["acc"], logs["acc_modal_0"], logs["acc_modal_1"]))
    cbs = [gate, Rec()]
    for c in cbs:
        c.set_model(model, ignore=False)
        c.set_optimizer(opt)
    M = Model_(model=model, optimizer=opt, loss_function=T.blend_loss, metrics=[T.acc],
               nummodalities=2)
    for c in cbs:
        c.set_model_pytoune(M)
    import io
    import contextlib
    with contextlib.redirect_stdout(io.StringIO()):
        M.train_loop(conv(train), valid_generator=conv(valid), test_generator=conv(test),
                     epochs=case["epochs"], steps_per_epoch=len(train),
                     validation_steps=len(valid), test_steps=len(test), callbacks=cbs)
    out = {"trace/steps": np.array(rec, dtype=np.float64)}
    model.eval()
    xe, _ = spec.model_inputs(ev)
    with torch.no_grad():
        lm, lo, _, _ = model(tt(xe))
    out["trace/eval_logits"] = lm.numpy()
    out["trace/eval_logits0"] = lo[0].numpy()
    out["trace/mmtm2_step"] = np.array(model.mmtm2.step)
    out["trace/mmtm4_ra_v"] = model.mmtm4.running_avg_weight_visual.numpy()
    out["trace/mmtm4_ra_s"] = model.mmtm4.running_avg_weight_skeleton.numpy()
    for n in spec.TRACE_PARAMS:
        out["trace/param." + n] = dict(model.named_parameters())[n].detach().numpy()
    return {k.replace("trace/", tag + "/"): v for k, v in out.items()}


def ddp_case(R):
    """F4: mean over shards of per-shard reference gradients (BN stats per shard)."""
    out = {}
    case = spec.DDP
    x, y = spec.model_inputs(case)
    grads = None
    for s in range(case["world"]):
        model = R.MMTM_MVCNN()
        weights.apply_to_module(model, seed=spec.SEED_MODEL)
        model.train(True)
        lo = case["B"] // case["world"]
        xs, ys = tt(x[s * lo:(s + 1) * lo]), tt(y[s * lo:(s + 1) * lo])
        _, outs, _, _ = model(xs)
        spec_blend_loss(outs, ys).backward()
        g = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
        grads = g if grads is None else {n: grads[n] + g[n] for n in g}
    names = list(grads)
    out["ddp/param_names"] = np.array(names)
    out["ddp/gn"] = np.array([float(((grads[n] / case["world"]) ** 2).sum()) for n in names])
    for n in names:
        idx = spec.sample_idx(n, grads[n].numel())
        out["ddp/gsample." + n] = (grads[n] / case["world"]).reshape(-1)[idx].numpy()
    return out


def cur_case(R):
    """F5: conditional-utilisation evaluation: recorded squeezes -> mmtm_off forward."""
    import src.balanced_mmtm as BM
    out = {}
    d = tempfile.mkdtemp()
    ev_dir, tr_dir = os.path.join(d, "eval"), os.path.join(d, "train")
    os.makedirs(ev_dir)
    os.makedirs(tr_dir)
    ev_hist, tr_hist = spec.cur_histories()
    with open(os.path.join(ev_dir, "history.pickle"), "wb") as f:
        pickle.dump(ev_hist, f)
    with open(os.path.join(tr_dir, "history.pickle"), "wb") as f:
        pickle.dump(tr_hist, f)
    w = BM.get_rescale_weights(ev_dir, tr_dir, validation=False, starting_mmtmindice=1,
                               mmtmpositions=4, device=None)
    for i in range(1, 4):
        out[f"cur/avg{i}_v"], out[f"cur/avg{i}_s"] = np.asarray(w[i][0]), np.asarray(w[i][1])
    model = R.MMTM_MVCNN(mmtm_off=True, mmtm_rescale_eval_file_path=ev_dir,
                         mmtm_rescale_training_file_path=tr_dir, device="cpu")
    weights.apply_to_module(model, seed=spec.SEED_MODEL)
    model.eval()
    x, _ = spec.model_inputs(spec.CUR)
    with torch.no_grad():
        lm, lo, _, _ = model(tt(x))
    out["cur/logits"], out["cur/logits0"], out["cur/logits1"] = lm.numpy(), lo[0].numpy(), lo[1].numpy()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    install_shims(args.ref)
    torch.manual_seed(0)
    import src.model as RM
    import src.balanced_mmtm as BM
    R = types.SimpleNamespace(MMTM_MVCNN=RM.MMTM_MVCNN, MMTM_mitigate=BM.MMTM_mitigate)
    blobs = {"mmtm": mmtm_cases(R), "model": model_cases(R), "trace": {**trace_case(R), **trace_case(R, spec.TRACE_GPU, spec.TRACE_GPU_EVAL, "trace_gpu")},
             "ddp": ddp_case(R), "cur": cur_case(R)}
    for k, v in blobs.items():
        path = os.path.join(HERE, f"golden_{k}.npz")
        np.savez_compressed(path, **v)
        print(f"wrote {path}: {len(v)} arrays, {os.path.getsize(path) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
