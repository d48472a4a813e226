"""Decision-level parity of the benchmarked bf16 gate with every outcome exercised
(VERDICT r03 missing #5 / next #3): the C2 step (B = 64 two-view 224x224 objects, bf16
trunk, hipGraph replay, on-device gate, lr 0.1, epsilon 0.02) against the fp32 oracle of
the reference step (/root/reference/src/callbacks.py:199-263, src/model.py:63-108,
train.py:23-29), teacher-forced AND steered:

before every deciding step the oracle runs the reference forward/backward from the HIP
run's current fp32 master weights on the same bf16-rounded batch; from its group sums the
test picks M accumulators (written into the device gate state and the oracle alike) that
put the oracle's d_BDR on a target taken from a schedule crossing epsilon in both signs -
so the trace holds no-curation, caring-0 and caring-1 decisions, most of them far enough
from +-epsilon to be judged.  The HIP step then adds its OWN bf16 group sums to the same M
and decides on the device.  Steered M sits in one bypass accumulator only (the main
accumulators stay 0), so the main-branch gradient sums of both views enter d_BDR with
their full bf16 error.

BAND is the bf16-vs-fp32 d_BDR noise the decisions are judged with: a step whose oracle
|d_BDR| lies within BAND of epsilon may legitimately decide either way; every other step
must decide identically (curate or not, and which modality).  That noise is the bf16 floor,
not a per-view defect (test_gpu_view_symmetry.py): PyTorch's own CPU bf16 autocast of the
oracle is as far from fp32 (gradient sums 6-8e-3 per branch, test_gpu_c2_bf16.py), i.e.
d_BDR moves by up to 0.434 x the four sums' errors ~ 1e-2.  The test measures that floor on
its first deciding steps (the oracle under CPU bf16 autocast from the same state and M) and
requires the HIP step's d_BDR noise to stay within it.  Epsilon is 0.02 here (the rule is
epsilon-independent; training_guided.gin's 0.01 would leave no room for a judged
no-curation step beside a 1e-2 band).
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B, H, EPS, WINDOW, LR = 64, 224, 0.02, 2, 0.1
BAND = 1e-2
# oracle d_BDR targets (cycled): both signs, inside and outside epsilon, a few near it
TARGETS = [0.040, -0.040, 0.0, 0.035, -0.035, 0.005, -0.005, 0.045, -0.045, 0.0, 0.032, -0.032, 0.022, -0.018,
           0.050, -0.050, 0.003, -0.003, 0.038, -0.038, 0.0, 0.042, -0.042, 0.008]
MIN_DECIDING = 22
FLOOR_STEPS = 6  # deciding steps on which the CPU bf16 floor is measured too


def _steer(r, target):
    """M = (bypass0, bypass1, main0, main1) with main = 0 such that
    log10((Mb0 + rb0) / rm0) - log10((Mb1 + rb1) / rm1) == target."""
    rb0, rb1, rm0, rm1 = r
    base = math.log10(rb0 / rm0) - math.log10(rb1 / rm1)
    if target >= base:
        return [rm0 * (rb1 / rm1) * 10.0 ** target - rb0, 0.0, 0.0, 0.0]
    return [0.0, rm1 * (rb0 / rm0) * 10.0 ** (-target) - rb1, 0.0, 0.0]


@pytest.fixture(scope="module")
def trace():
    return _trace(EPS, TARGETS, MIN_DECIDING, FLOOR_STEPS)


# training_guided.gin's own epsilon (configs/training_guided.gin:14): 0.01.  With the 1e-2 bf16
# band no no-curation step can be judged (|d_BDR| < 0.01 lies inside the band of +-0.01), so the
# targets put most steps far beyond it in both signs (judged: curate + which modality) and the rest
# near 0 / near +-epsilon (reported: how often the bf16 step still matches there)
EPS_GUIDED = 0.01
TARGETS_GUIDED = [0.030, -0.030, 0.0, 0.025, -0.025, 0.012, -0.012, 0.040, -0.040, 0.004, 0.022, -0.022, 0.008,
                  -0.006, 0.050, -0.050]
MIN_DECIDING_GUIDED = 16


@pytest.fixture(scope="module")
def trace_guided():
    return _trace(EPS_GUIDED, TARGETS_GUIDED, MIN_DECIDING_GUIDED, 0)


def _trace(EPS, TARGETS, MIN_DECIDING, FLOOR_STEPS):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    from greedy_multimodal_learning_amd.engine import BalancedStep
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    from oracle import gating_ref, model_ref, weights
    dev = torch.device("cuda:0")
    torch.set_num_threads(max(1, min(32, torch.get_num_threads())))
    model = weights.apply_to_module(MMTM_MVCNN(), seed=5).to(dev)
    gate = Bias_Mitigation_Strong(epsilon=EPS, curation_windowsize=WINDOW, branchnames=["net_view_0", "net_view_1"],
                                  starting_epoch=1)
    step = BalancedStep(model, lr=LR, gate=gate, graphs=True)
    step.on_epoch_begin(1)
    assert step.device_gate and step.graphs
    g = torch.Generator().manual_seed(91)
    batches = []
    for _ in range(4):
        buf = torch.randn(2, B, H, H, 3, generator=g).bfloat16()
        batches.append((buf, torch.randint(0, 40, (B,), generator=g)))
    dbat = [(b.to(dev).permute(1, 0, 4, 2, 3), y.to(dev)) for b, y in batches]
    oracle = model_ref.MMTM_MVCNN_Ref()
    rows, t, k = [], 0, 0
    while len(rows) < MIN_DECIDING:
        st = step.sync_gate()
        x, y = dbat[t % 4]
        if st["curation_mode"]:  # inside a curation window: no decision this step
            step(x, y)
            t += 1
            continue
        oracle.load_state_dict({n: p.detach().float().contiguous().cpu() for n, p in model.named_parameters()},
                               strict=False)
        oracle.zero_grad(set_to_none=True)
        oracle.train(True)
        buf, yc = batches[t % 4]
        _, outs, _, _ = oracle(buf.float().permute(1, 0, 4, 2, 3).contiguous())
        gating_ref.blend_loss(outs, yc).backward()
        s = gating_ref.group_sums([(n, p, p.grad) for n, p in oracle.named_parameters()])
        r = [s["gn_bypass"][0] / s["wn_bypass"][0], s["gn_bypass"][1] / s["wn_bypass"][1],
             s["gn_main"][0] / s["wn_main"][0], s["gn_main"][1] / s["wn_main"][1]]
        M = _steer(r, TARGETS[k % len(TARGETS)])
        k += 1
        gs = step.gate_struct()
        for i in range(4):
            gs.M[i] = M[i]
        step.set_gate_struct(gs)
        bdr = gating_ref.BDRState(EPS, WINDOW)
        bdr.M_bypass, bdr.M_main = [M[0], M[1]], [M[2], M[3]]
        d_o = float(bdr.update(s))
        d_b = None
        if len(rows) < FLOOR_STEPS:  # the bf16 floor: the same step under CPU bf16 autocast
            oracle.zero_grad(set_to_none=True)
            with torch.autocast("cpu", dtype=torch.bfloat16):
                _, outs16, _, _ = oracle(buf.float().permute(1, 0, 4, 2, 3).contiguous())
            gating_ref.blend_loss([o_.float() for o_ in outs16], yc).backward()
            s16 = gating_ref.group_sums([(n, p, p.grad) for n, p in oracle.named_parameters()])
            b16 = gating_ref.BDRState(EPS, WINDOW)
            b16.M_bypass, b16.M_main = [M[0], M[1]], [M[2], M[3]]
            d_b = float(b16.update(s16))
        step(x, y)
        t += 1
        after = step.sync_gate()
        dec_o = (abs(d_o) > EPS, (1 if d_o < 0 else 0) if abs(d_o) > EPS else 0)
        dec_h = (bool(after["curation_mode"]), after["caring_modality"] if after["curation_mode"] else 0)
        rows.append((t - 1, after["d_BDR"], d_o, dec_h, dec_o, d_b))
        print(f"step {t - 1:2d}: target {TARGETS[(k - 1) % len(TARGETS)]:+.4f} d_BDR hip {after['d_BDR']:+.5f} "
              f"oracle {d_o:+.5f} |diff| {abs(after['d_BDR'] - d_o):.2e}"
              + (f" (cpu bf16 {d_b:+.5f}, |diff| {abs(d_b - d_o):.2e})" if d_b is not None else "")
              + f" decision hip {dec_h} oracle {dec_o}", flush=True)
    return rows


def test_steered_gate_decisions_vs_oracle(trace):
    rows = trace
    diff = np.array([abs(r[1] - r[2]) for r in rows])
    floor = np.array([abs(r[5] - r[2]) for r in rows if r[5] is not None])
    print(f"d_BDR |hip - oracle| over {len(rows)} deciding steps: median {np.median(diff):.2e} "
          f"p90 {np.percentile(diff, 90):.2e} max {diff.max():.2e}; CPU bf16 floor over {len(floor)}: "
          f"median {np.median(floor):.2e} max {floor.max():.2e}")
    assert diff.max() < BAND, "bf16 d_BDR noise above the band the decisions are judged with"
    # the HIP step is no noisier than PyTorch's own bf16 (medians: single steps scatter)
    assert np.median(diff) <= 2 * max(np.median(floor), 1e-3), (np.median(diff), np.median(floor))
    clear = [r for r in rows if abs(abs(r[2]) - EPS) > BAND]
    assert len(clear) >= len(rows) // 2, (len(clear), len(rows))
    outcomes = {r[4] for r in clear}
    assert {(False, 0), (True, 0), (True, 1)} <= outcomes, outcomes
    for t, dh, do, dec_h, dec_o, _ in clear:
        assert dec_h == dec_o, (t, dh, do, dec_h, dec_o)
    agree = sum(r[3] == r[4] for r in rows)
    print(f"decisions identical on {agree}/{len(rows)} deciding steps ({len(clear)} outside the band)")


def test_steered_gate_decisions_at_guided_epsilon(trace_guided):
    """The same teacher-forced, steered C2 bf16 step at training_guided.gin's epsilon = 0.01: every
    step whose oracle d_BDR lies outside the bf16 band around +-epsilon (|d| > 0.02 here) must
    curate the same modality; steps inside the band (every no-curation step at this epsilon)
    are reported with the fraction that still decides like the fp32 reference."""
    rows = trace_guided
    eps = EPS_GUIDED
    clear = [r for r in rows if abs(abs(r[2]) - eps) > BAND]
    inside = [r for r in rows if abs(abs(r[2]) - eps) <= BAND]
    assert len(clear) >= len(rows) // 2, (len(clear), len(rows))
    assert {(True, 0), (True, 1)} <= {r[4] for r in clear}
    for t, dh, do, dec_h, dec_o, _ in clear:
        assert dec_h == dec_o, (t, dh, do, dec_h, dec_o)
    agree_in = sum(r[3] == r[4] for r in inside)
    diff = np.array([abs(r[1] - r[2]) for r in rows])
    print(f"epsilon {eps}: decisions identical on {len(clear)}/{len(clear)} steps outside the band and "
          f"{agree_in}/{len(inside)} inside it ({sum(r[4][0] is False for r in inside)} of those no-curation in the "
          f"fp32 reference); d_BDR |hip - oracle| median {np.median(diff):.2e} max {diff.max():.2e}")
    assert diff.max() < BAND
