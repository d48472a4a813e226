"""Pin the CPU oracle against the reference's own outputs (tests/golden/*.npz).

CPU only.  Every fixture was produced by importing the reference
(tests/golden/make_golden.py); inputs are regenerated from tests/golden/spec.py.
Tolerance: fp32 restatement of identical arithmetic -> rtol 1e-4 (north_star).
"""
import os
import pickle
import tempfile

import numpy as np
import pytest
import torch

import spec
from helpers import close
from oracle import cur_ref, gating_ref, loop_ref, mmtm_ref, model_ref, step_ref, weights

tt = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731


def _mmtm_kwargs(case):
    mode = case["mode"]
    avg = spec.mmtm_avg(case)
    return dict(return_scale=True, return_squeezed_mps=(mode == "normal"),
                turnoff_cross_modal_flow=(mode == "turnoff"),
                average_squeezemaps=[tt(avg[0]), tt(avg[1])] if mode == "turnoff" else None,
                curation_mode=mode.startswith("cur"),
                caring_modality=int(mode[-1]) if mode.startswith("cur") else 0)


@pytest.mark.parametrize("case", spec.MMTM_CASES, ids=lambda c: c["id"])
def test_oracle_mmtm(golden, case):
    fix = golden["mmtm"]
    C = case["C"]
    m = mmtm_ref.MMTMRef(C, C, 4, SEonly=case.get("SEonly", False),
                         shareweight=case.get("shareweight", False))
    weights.apply_to_module(m, seed=spec.SEED_MMTM)
    for k in range(case.get("warm", 0)):
        wv, ws = spec.mmtm_warm_inputs(case, k)
        with torch.no_grad():
            m(tt(wv), tt(ws))
    xv, xs, dyv, dys = spec.mmtm_inputs(case)
    Xv, Xs = tt(xv).requires_grad_(True), tt(xs).requires_grad_(True)
    Yv, Ys, sc, sq = m(Xv, Xs, **_mmtm_kwargs(case))
    ((Yv * tt(dyv)).sum() + (Ys * tt(dys)).sum()).backward()
    p = case["id"] + "/"
    close(fix, p + "Yv", Yv.detach())
    close(fix, p + "Ys", Ys.detach())
    close(fix, p + "ev", sc[0])
    close(fix, p + "es", sc[1])
    if sq is not None:
        close(fix, p + "sqv", sq[0])
        close(fix, p + "sqs", sq[1])
    close(fix, p + "dXv", Xv.grad)
    close(fix, p + "dXs", Xs.grad)
    for n, prm in m.named_parameters():
        g = prm.grad if prm.grad is not None else torch.full(prm.shape, float("nan"))
        close(fix, p + "grad." + n, g.numpy(), rtol=1e-4, atol=1e-5)
    close(fix, p + "ra_v", m.running_avg_weight_visual)
    close(fix, p + "ra_s", m.running_avg_weight_skeleton)
    assert int(fix[p + "step"]) == m.step


def test_oracle_mmtm_squeeze_error_in_turnoff():
    """Reference quirk: return_squeezed_mps in turn-off mode raises (`:123-124`)."""
    m = mmtm_ref.MMTMRef(8, 8, 4)
    x = torch.randn(2, 8, 2, 2)
    with pytest.raises(UnboundLocalError):
        m(x, x, return_squeezed_mps=True, turnoff_cross_modal_flow=True,
          average_squeezemaps=[torch.zeros(8), torch.zeros(8)])


def _model():
    m = model_ref.MMTM_MVCNN_Ref(saving_mmtm_scales=True, saving_mmtm_squeeze_array=True)
    return weights.apply_to_module(m, seed=spec.SEED_MODEL)


@pytest.mark.parametrize("case", spec.MODEL_CASES, ids=lambda c: c["id"])
def test_oracle_model(golden, case):
    fix = golden["model"]
    p = case["id"] + "/"
    m = _model()
    m.train(True)
    x, y = spec.model_inputs(case)
    mean, outs, scales, sqs = m(tt(x), curation_mode=case.get("cur", False),
                                caring_modality=case.get("caring", None))
    loss = gating_ref.blend_loss(outs, tt(y))
    loss.backward()
    close(fix, p + "logits", mean.detach(), rtol=1e-4, atol=1e-4)
    close(fix, p + "logits0", outs[0].detach(), rtol=1e-4, atol=1e-4)
    close(fix, p + "logits1", outs[1].detach(), rtol=1e-4, atol=1e-4)
    assert abs(float(loss.detach()) - float(fix[p + "loss"])) < 1e-4 * abs(float(fix[p + "loss"]))
    for i in range(3):
        close(fix, p + f"scale{i}_v", scales[i][0], atol=1e-5)
        close(fix, p + f"sq{i}_s", sqs[i][1], atol=1e-5)
    names = [n for n, _ in m.named_parameters()]
    assert names == list(fix[p + "param_names"])
    gn = np.array([float((q.grad ** 2).sum()) if q.grad is not None else 0.0
                   for _, q in m.named_parameters()])
    np.testing.assert_allclose(gn, fix[p + "gn"], rtol=2e-4, atol=1e-9)
    for n, q in m.named_parameters():
        if q.grad is not None and (p + "gsample." + n) in fix.files:
            idx = spec.sample_idx(n, q.numel())
            np.testing.assert_allclose(q.grad.reshape(-1)[idx].numpy(), fix[p + "gsample." + n],
                                       rtol=1e-3, atol=1e-6, err_msg=n)
    if (p + "d_BDR") in fix.files:
        named = [(n, q, q.grad) for n, q in m.named_parameters()]
        st = gating_ref.BDRState(0.01, 5)
        d = st.update(gating_ref.group_sums(named))
        assert abs(d - float(fix[p + "d_BDR"])) < 1e-5
    close(fix, p + "bn_rm", m.net_view_0.layer2[0].bn1.running_mean, atol=1e-5)
    close(fix, p + "bn_rv", m.net_view_1.layer4[1].bn2.running_var, atol=1e-5)


@pytest.mark.parametrize("tag", ["trace", "trace_gpu"])
def test_oracle_trace(golden, tag):
    """Whole guided run (3 epochs x 4 steps) through the reference loop order."""
    fix = golden["trace"]
    t = spec.TRACE if tag == "trace" else spec.TRACE_GPU
    ev = spec.TRACE_EVAL if tag == "trace" else spec.TRACE_GPU_EVAL
    m = weights.apply_to_module(model_ref.MMTM_MVCNN_Ref(), seed=spec.SEED_MODEL)
    gate = gating_ref.BDRState(t["epsilon"], t["window"], t["starting_epoch"])
    step = step_ref.RefStep(m, lr=t["lr"], gate=gate)
    train, valid, test = spec.trace_loaders(t)
    conv = lambda L: [(i, tt(x), tt(y)) for i, x, y in L]  # noqa: E731
    rows = np.array(loop_ref.run(m, step, gate, conv(train), conv(valid), conv(test), t["epochs"]),
                    dtype=np.float64)
    ref = fix[tag + "/steps"]
    assert rows.shape == ref.shape
    np.testing.assert_allclose(rows[:, 0], ref[:, 0], rtol=1e-4)       # loss
    np.testing.assert_allclose(rows[:, 1], ref[:, 1], atol=1e-5)       # d_BDR
    np.testing.assert_array_equal(rows[:, 2:4], ref[:, 2:4])           # decisions
    np.testing.assert_allclose(rows[:, 4:], ref[:, 4:], atol=1e-9)     # accuracies
    m.eval()
    xe, _ = spec.model_inputs(ev)
    with torch.no_grad():
        lm, lo, _, _ = m(tt(xe))
    close(fix, tag + "/eval_logits", lm, rtol=1e-3, atol=1e-3)
    assert int(fix[tag + "/mmtm2_step"]) == m.mmtm2.step
    close(fix, tag + "/mmtm4_ra_v", m.mmtm4.running_avg_weight_visual, atol=1e-5)
    close(fix, tag + "/mmtm4_ra_s", m.mmtm4.running_avg_weight_skeleton, atol=1e-5)
    P = dict(m.named_parameters())
    for n in spec.TRACE_PARAMS:
        close(fix, tag + "/param." + n, P[n].detach(), rtol=1e-3, atol=1e-4)


def test_oracle_ddp_mean_of_shards(golden):
    fix = golden["ddp"]
    c = spec.DDP
    x, y = spec.model_inputs(c)
    acc = None
    lo = c["B"] // c["world"]
    for s in range(c["world"]):
        m = weights.apply_to_module(model_ref.MMTM_MVCNN_Ref(), seed=spec.SEED_MODEL)
        _, outs, _, _ = m(tt(x[s * lo:(s + 1) * lo]))
        gating_ref.blend_loss(outs, tt(y[s * lo:(s + 1) * lo])).backward()
        g = {n: q.grad.clone() for n, q in m.named_parameters()}
        acc = g if acc is None else {n: acc[n] + g[n] for n in g}
    names = list(fix["ddp/param_names"])
    gn = np.array([float(((acc[n] / c["world"]) ** 2).sum()) for n in names])
    np.testing.assert_allclose(gn, fix["ddp/gn"], rtol=2e-4, atol=1e-9)


def test_oracle_cur(golden):
    fix = golden["cur"]
    ev, tr = spec.cur_histories()
    d = tempfile.mkdtemp()
    for sub, h in (("eval", ev), ("train", tr)):
        os.makedirs(os.path.join(d, sub))
        with open(os.path.join(d, sub, "history.pickle"), "wb") as f:
            pickle.dump(h, f)
    w = cur_ref.rescale_weights(os.path.join(d, "eval"), os.path.join(d, "train"))
    assert w[0] is None
    for i in range(1, 4):
        close(fix, f"cur/avg{i}_v", w[i][0], atol=1e-6)
        close(fix, f"cur/avg{i}_s", w[i][1], atol=1e-6)
    m = model_ref.MMTM_MVCNN_Ref(mmtm_off=True,
                                 mmtm_rescale=[None] + [[tt(a), tt(b)] for a, b in w[1:]])
    weights.apply_to_module(m, seed=spec.SEED_MODEL)
    m.eval()
    x, _ = spec.model_inputs(spec.CUR)
    with torch.no_grad():
        lm, lo, _, _ = m(tt(x))
    close(fix, "cur/logits", lm, rtol=1e-4, atol=1e-4)
    close(fix, "cur/logits0", lo[0], rtol=1e-4, atol=1e-4)
    close(fix, "cur/logits1", lo[1], rtol=1e-4, atol=1e-4)
