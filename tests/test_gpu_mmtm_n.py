"""N-modality MMTM on the GPU.

* N = 2: MMTM_N carrying the reference module's weights must reproduce the
  reference's golden MMTM fixtures (normal / curation / turn-off cases), rtol 1e-4.
* N = 3, 4: no reference exists beyond two modalities ("parity unpinned" w.r.t.
  the reference); checked against a plain PyTorch fp32 autograd restatement of
  the documented N-way rule in this file, fwd + all gradients, rtol 1e-4.
* Model level: MMTM_MVCNN_N(num_views=2) == MMTM_MVCNN with the same weights; a
  4-view training step through the engine with the N-branch gate.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import spec
from helpers import close
from oracle import weights

pytestmark = pytest.mark.gpu
tt = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731

N2_CASES = [c for c in spec.MMTM_CASES if not c.get("SEonly") and not c.get("shareweight")]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _from_reference_module(C, dev):
    from greedy_multimodal_learning_amd.balanced_mmtm import MMTM_mitigate
    from greedy_multimodal_learning_amd.mmtm_n import MMTM_N
    ref = MMTM_mitigate(C, C, 4)
    weights.apply_to_module(ref, seed=spec.SEED_MMTM)
    m = MMTM_N([C, C], 4)
    with torch.no_grad():
        m.fc_squeeze.weight.copy_(ref.fc_squeeze.weight)
        m.fc_squeeze.bias.copy_(ref.fc_squeeze.bias)
        m.fc_excite[0].weight.copy_(ref.fc_visual.weight)
        m.fc_excite[0].bias.copy_(ref.fc_visual.bias)
        m.fc_excite[1].weight.copy_(ref.fc_skeleton.weight)
        m.fc_excite[1].bias.copy_(ref.fc_skeleton.bias)
    return m.to(dev)


@pytest.mark.parametrize("case", N2_CASES, ids=lambda c: c["id"])
def test_mmtm_n2_matches_reference_fixtures(golden, dev, case):
    fix = golden["mmtm"]
    m = _from_reference_module(case["C"], dev)
    prep = lambda a, g=False: tt(a).to(dev).requires_grad_(g)  # noqa: E731
    for k in range(case.get("warm", 0)):
        wv, ws = spec.mmtm_warm_inputs(case, k)
        with torch.no_grad():
            m([prep(wv), prep(ws)])
    xv, xs, dyv, dys = spec.mmtm_inputs(case)
    Xv, Xs = prep(xv, True), prep(xs, True)
    mode = case["mode"]
    kw = dict(return_scale=True, return_squeezed_mps=(mode == "normal"))
    if mode == "turnoff":
        avg = spec.mmtm_avg(case)
        kw.update(turnoff_cross_modal_flow=True, average_squeezemaps=[tt(avg[0]), tt(avg[1])])
    if mode.startswith("cur"):
        kw.update(curation_mode=True, caring_modality=int(mode[-1]))
    (Yv, Ys), sc, sq = m([Xv, Xs], **kw)
    torch.autograd.backward([Yv, Ys], [prep(dyv), prep(dys)])
    p = case["id"] + "/"
    f = lambda t: t.detach().float().cpu()  # noqa: E731
    close(fix, p + "Yv", f(Yv))
    close(fix, p + "Ys", f(Ys))
    close(fix, p + "ev", sc[0])
    close(fix, p + "es", sc[1])
    if sq is not None:
        close(fix, p + "sqv", sq[0])
        close(fix, p + "sqs", sq[1])
    close(fix, p + "dXv", f(Xv.grad))
    close(fix, p + "dXs", f(Xs.grad))
    names = {"fc_squeeze.weight": m.fc_squeeze.weight, "fc_squeeze.bias": m.fc_squeeze.bias,
             "fc_visual.weight": m.fc_excite[0].weight, "fc_visual.bias": m.fc_excite[0].bias,
             "fc_skeleton.weight": m.fc_excite[1].weight, "fc_skeleton.bias": m.fc_excite[1].bias}
    for n, prm in names.items():
        g = f(prm.grad) if prm.grad is not None else torch.full(prm.shape, float("nan"))
        close(fix, p + "grad." + n, g.numpy(), rtol=1e-4, atol=1e-5)
    close(fix, p + "ra_v", f(m.running_avg[0]))


def _torch_nway(xs, Wsq, bsq, We, be, ra, step, curation, caring, avg=None):
    """fp32 autograd restatement of MMTM_N (documented N-way rule)."""
    N = len(xs)
    sqs = [x.flatten(2).mean(-1) for x in xs]
    sq = torch.cat(sqs, 1)
    if avg is None:
        z = F.relu(F.linear(sq, Wsq, bsq))
        zs = [z] * N
    else:
        offs = np.cumsum([0] + [x.shape[1] for x in xs])
        zs = []
        for i in range(N):
            parts = [sqs[j] if j == i else avg[offs[j]:offs[j + 1]].expand(xs[0].shape[0], -1) for j in range(N)]
            zs.append(F.relu(F.linear(torch.cat(parts, 1), Wsq, bsq)))
    es = [torch.sigmoid(F.linear(zs[i], We[i], be[i])) for i in range(N)]
    m0 = es[0].detach().mean(0)
    ra_new = [(m0 + r * step) / (step + 1) for r in ra]
    ys = []
    for i in range(N):
        s = ra_new[i].expand_as(es[i]) if (curation and i == caring) else es[i]
        ys.append(xs[i] * s[:, :, None, None])
    return ys, es, ra_new


@pytest.mark.parametrize("N,curation,caring,turnoff", [(3, False, 0, False), (4, False, 0, False),
                                                       (4, True, 2, False), (3, True, 0, False),
                                                       (4, False, 0, True)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_mmtm_n_vs_torch(dev, N, curation, caring, turnoff, dtype):
    from greedy_multimodal_learning_amd.mmtm_n import MMTM_N
    g = torch.Generator().manual_seed(N * 10 + caring)
    B, C, H, W = 3, 128, 5, 5
    m = MMTM_N([C] * N, 4).to(dev)
    xs = [torch.randn(B, C, H, W, generator=g).to(dev).to(dtype) for _ in range(N)]
    dys = [torch.randn(B, C, H, W, generator=g).to(dev).to(dtype) for _ in range(N)]
    ra0 = [torch.rand(C, generator=g).to(dev) for _ in range(N)]
    m.running_avg = [r.clone() for r in ra0]
    m.step = 3
    avg = torch.randn(N * C, generator=g).to(dev) if turnoff else None
    xa = [x.clone().requires_grad_(True) for x in xs]
    kw = dict(curation_mode=curation, caring_modality=caring)
    if turnoff:
        kw.update(turnoff_cross_modal_flow=True, average_squeezemaps=[avg[i * C:(i + 1) * C] for i in range(N)])
    ys, sc, _ = m(xa, return_scale=True, **kw)
    torch.autograd.backward(ys, dys)
    # reference on the (rounded) inputs in fp32
    xr = [x.float().clone().requires_grad_(True) for x in xs]
    Wsq = m.fc_squeeze.weight.detach().clone().requires_grad_(True)
    bsq = m.fc_squeeze.bias.detach().clone().requires_grad_(True)
    We = [e.weight.detach().clone().requires_grad_(True) for e in m.fc_excite]
    be = [e.bias.detach().clone().requires_grad_(True) for e in m.fc_excite]
    yr, er, rr = _torch_nway(xr, Wsq, bsq, We, be, ra0, 3, curation, caring, avg)
    torch.autograd.backward(yr, [d.float() for d in dys])
    tol = dict(rtol=1e-4, atol=1e-5) if dtype == torch.float32 else dict(rtol=2e-2, atol=2e-2)
    for i in range(N):
        torch.testing.assert_close(ys[i].float(), yr[i], **tol)
        torch.testing.assert_close(sc[i].to(dev), er[i], **tol)
        torch.testing.assert_close(xa[i].grad.float(), xr[i].grad, **tol)
        torch.testing.assert_close(m.running_avg[i], rr[i], rtol=1e-5, atol=1e-6)
        if curation and i == caring:
            assert m.fc_excite[i].weight.grad is None
        else:
            torch.testing.assert_close(m.fc_excite[i].weight.grad, We[i].grad, **tol)
            torch.testing.assert_close(m.fc_excite[i].bias.grad, be[i].grad, **tol)
    torch.testing.assert_close(m.fc_squeeze.weight.grad, Wsq.grad, **tol)
    torch.testing.assert_close(m.fc_squeeze.bias.grad, bsq.grad, **tol)
    assert m.step == 4


def test_model_n2_equals_reference_model(dev):
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN, MMTM_MVCNN_N
    torch.manual_seed(0)
    a = MMTM_MVCNN(nclasses=40).to(dev)
    b = MMTM_MVCNN_N(nclasses=40, num_views=2).to(dev)
    sa = a.state_dict()
    rename = {"fc_visual": "fc_excite.0", "fc_skeleton": "fc_excite.1"}
    sb = {}
    for k, v in sa.items():
        for old, new in rename.items():
            k = k.replace(old, new)
        sb[k] = v
    b.load_state_dict(sb, strict=True)
    x = torch.randn(2, 2, 3, 64, 64, device=dev)
    la, oa, _, _ = a(x)
    lb, ob, _, _ = b(x)
    torch.testing.assert_close(lb, la, rtol=1e-5, atol=1e-5)
    for u, v in zip(ob, oa):
        torch.testing.assert_close(u, v, rtol=1e-5, atol=1e-5)


def test_four_view_engine_step_with_n_branch_gate(dev):
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    from greedy_multimodal_learning_amd.engine import BalancedStep
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN_N
    torch.manual_seed(1)
    m = MMTM_MVCNN_N(nclasses=40, num_views=4).to(dev)
    gate = Bias_Mitigation_Strong(epsilon=1e-6, curation_windowsize=2, branchnames=m.branch_names(),
                                  starting_epoch=1, MMTMnames=m.mmtm_names())
    step = BalancedStep(m, lr=0.01, gate=gate, branchnames=m.branch_names(), MMTMnames=m.mmtm_names())
    step.on_epoch_begin(1)
    x = torch.randn(4, 4, 3, 64, 64, device=dev)
    y = torch.randint(0, 40, (4,), device=dev)
    loss = step(x, y)
    assert torch.isfinite(loss)
    assert step.device_gate and step.gate_n  # the N-branch on-device gate (gm_gate_state_n)
    step.sync_gate()  # the host mirrors (gate.BDR, flags) are filled on request
    bdr = list(gate.BDR)
    assert len(bdr) == 4 and all(np.isfinite(bdr))
    # epsilon 1e-6: the first decision curates, caring for the argmax-BDR branch
    assert step.flags.curation_mode and step.flags.caring_modality == int(np.argmax(bdr))
    for _ in range(3):
        assert torch.isfinite(step(x, y))
