"""MMTM fusion op on the GPU: HIP path vs the reference's golden outputs and the oracle.

fp32 (NCHW and channels_last): rtol 1e-4 against the reference fixtures
(north_star tolerance).  bf16 activations: compared with the fp32 oracle run on
the same bf16-rounded inputs, tolerance 2e-2 relative (bf16 has 8 mantissa bits;
the FC chain itself is fp32).
"""
import numpy as np
import pytest
import torch

import spec
from helpers import close
from oracle import mmtm_ref, weights

pytestmark = pytest.mark.gpu

tt = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _kwargs(case, dev):
    mode = case["mode"]
    avg = spec.mmtm_avg(case)
    return dict(return_scale=True, return_squeezed_mps=(mode == "normal"),
                turnoff_cross_modal_flow=(mode == "turnoff"),
                average_squeezemaps=[tt(avg[0]).to(dev), tt(avg[1]).to(dev)] if mode == "turnoff" else None,
                curation_mode=mode.startswith("cur"),
                caring_modality=int(mode[-1]) if mode.startswith("cur") else 0)


def _run(case, dev, dtype=torch.float32, channels_last=False):
    from greedy_multimodal_learning_amd.balanced_mmtm import MMTM_mitigate
    C = case["C"]
    m = MMTM_mitigate(C, C, 4, SEonly=case.get("SEonly", False),
                      shareweight=case.get("shareweight", False))
    weights.apply_to_module(m, seed=spec.SEED_MMTM)
    m = m.to(dev)
    fmt = torch.channels_last if channels_last else torch.contiguous_format

    def prep(a, grad=False):
        t = tt(a).to(dev).to(dtype).contiguous(memory_format=fmt)
        return t.requires_grad_(grad)
    for k in range(case.get("warm", 0)):
        wv, ws = spec.mmtm_warm_inputs(case, k)
        with torch.no_grad():
            m(prep(wv), prep(ws))
    xv, xs, dyv, dys = spec.mmtm_inputs(case)
    Xv, Xs = prep(xv, True), prep(xs, True)
    Yv, Ys, sc, sq = m(Xv, Xs, **_kwargs(case, dev))
    torch.autograd.backward([Yv, Ys], [prep(dyv), prep(dys)])
    return m, Xv, Xs, Yv, Ys, sc, sq


@pytest.mark.parametrize("channels_last", [False, True], ids=["nchw", "nhwc"])
@pytest.mark.parametrize("case", spec.MMTM_CASES, ids=lambda c: c["id"])
def test_mmtm_fp32_vs_reference(golden, dev, case, channels_last):
    fix = golden["mmtm"]
    m, Xv, Xs, Yv, Ys, sc, sq = _run(case, dev, torch.float32, channels_last)
    p = case["id"] + "/"
    f = lambda t: t.detach().float().cpu().contiguous()  # noqa: E731
    close(fix, p + "Yv", f(Yv))
    close(fix, p + "Ys", f(Ys))
    close(fix, p + "ev", sc[0])
    close(fix, p + "es", sc[1])
    if sq is not None:
        close(fix, p + "sqv", sq[0])
        close(fix, p + "sqs", sq[1])
    close(fix, p + "dXv", f(Xv.grad))
    close(fix, p + "dXs", f(Xs.grad))
    for n, prm in m.named_parameters():
        g = f(prm.grad) if prm.grad is not None else torch.full(prm.shape, float("nan"))
        close(fix, p + "grad." + n, g.numpy(), rtol=1e-4, atol=1e-5)
    close(fix, p + "ra_v", f(m.running_avg_weight_visual))
    close(fix, p + "ra_s", f(m.running_avg_weight_skeleton))
    assert int(fix[p + "step"]) == m.step


@pytest.mark.parametrize("channels_last", [False, True], ids=["nchw", "nhwc"])
@pytest.mark.parametrize("case", [c for c in spec.MMTM_CASES if c["id"] in
                                  ("n128", "n512r", "n128r", "c0", "c1", "off", "se", "sw")],
                         ids=lambda c: c["id"])
def test_mmtm_bf16_vs_oracle(dev, case, channels_last):
    m, Xv, Xs, Yv, Ys, sc, sq = _run(case, dev, torch.bfloat16, channels_last)
    # oracle on the same bf16-rounded inputs, in fp32
    C = case["C"]
    o = mmtm_ref.MMTMRef(C, C, 4, SEonly=case.get("SEonly", False),
                         shareweight=case.get("shareweight", False))
    weights.apply_to_module(o, seed=spec.SEED_MMTM)
    r = lambda a: tt(a).to(torch.bfloat16).float()  # noqa: E731
    for k in range(case.get("warm", 0)):
        wv, ws = spec.mmtm_warm_inputs(case, k)
        with torch.no_grad():
            o(r(wv), r(ws))
    xv, xs, dyv, dys = spec.mmtm_inputs(case)
    Ov, Os = r(xv).requires_grad_(True), r(xs).requires_grad_(True)
    kw = _kwargs(case, "cpu")
    RYv, RYs, rsc, _ = o(Ov, Os, **kw)
    torch.autograd.backward([RYv, RYs], [r(dyv), r(dys)])
    cmp = lambda a, b, tol=2e-2: np.testing.assert_allclose(  # noqa: E731
        a.detach().float().cpu().numpy(), b.detach().float().numpy(), rtol=tol,
        atol=tol * float(b.detach().abs().max()))
    cmp(Yv, RYv)
    cmp(Ys, RYs)
    cmp(sc[0], rsc[0], 1e-4)
    cmp(sc[1], rsc[1], 1e-4)
    cmp(Xv.grad, Ov.grad)
    cmp(Xs.grad, Os.grad)
    for (n, pg), (_, po) in zip(m.named_parameters(), o.named_parameters()):
        assert (pg.grad is None) == (po.grad is None), n
        if pg.grad is not None:
            cmp(pg.grad, po.grad, 2e-2)


def test_mmtm_rejects_cpu_tensors():
    from greedy_multimodal_learning_amd.balanced_mmtm import MMTM_mitigate
    from greedy_multimodal_learning_amd._lib import GreedyMMLError
    m = MMTM_mitigate(8, 8, 4)
    x = torch.randn(2, 8, 2, 2)
    with pytest.raises(GreedyMMLError):
        m(x, x)


def test_mmtm_turnoff_squeeze_raises(dev):
    from greedy_multimodal_learning_amd.balanced_mmtm import MMTM_mitigate
    m = MMTM_mitigate(8, 8, 4).to(dev)
    x = torch.randn(2, 8, 2, 2, device=dev)
    with pytest.raises(UnboundLocalError):
        m(x, x, return_squeezed_mps=True, turnoff_cross_modal_flow=True,
          average_squeezemaps=[torch.zeros(8, device=dev), torch.zeros(8, device=dev)])


@pytest.mark.parametrize("form", [(256, 4), (-256, 4), (-256, 8), (1024, 4), (-1024, 4)],
                         ids=lambda f: f"t{abs(f[0])}u{f[1]}{'nt' if f[0] < 0 else ''}")
@pytest.mark.parametrize("C,H,B", [(128, 28, 64), (256, 14, 64), (512, 7, 64), (128, 28, 256), (64, 9, 5)])
def test_squeeze_forms_vs_torch(dev, form, C, H, B):
    """Every form of the NHWC bf16 squeeze (k_colreduce_nhwc: threads x pixels in flight,
    nontemporal loads) against the fp32 torch mean over the same bf16 activations, both
    modalities in one launch, incl. a ragged map (9x9) and the north-star batch 256."""
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import ops
    lib = L.load()
    g = torch.Generator(device=dev).manual_seed(C + H + B)
    xs = [torch.randn(B, C, H, H, device=dev, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
          for _ in range(2)]
    sq = torch.empty(B, 2 * C, device=dev)
    try:
        L.check(lib.gm_mmtm_set_reduce_form(form[0], form[1]), "form")
        ops.spatial_reduce([dict(x=xs[0], C=C, HW=H * H, out=sq, ld_out=2 * C, scale=1.0 / (H * H)),
                            dict(x=xs[1], C=C, HW=H * H, out=sq, out_off=C, ld_out=2 * C, scale=1.0 / (H * H))],
                           B, L.GM_BF16, L.GM_NHWC, dev)
        torch.cuda.synchronize()
    finally:
        L.check(lib.gm_mmtm_set_reduce_form(-256, 4), "form")
    ref = torch.cat([x.float().mean(dim=(2, 3)) for x in xs], dim=1)
    torch.testing.assert_close(sq, ref, rtol=1e-5, atol=1e-6)
