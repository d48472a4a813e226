"""The benchmarked workload itself, checked for correctness: config C2 (B = 64 two-view
224x224 objects, bf16 trunk, BalancedStep with hipGraph replay and the on-device gate
- exactly what bench.py times) against the oracle's fp32 CPU restatement of the
reference step (/root/reference/src/model.py:63-108, train.py:23-29,
src/callbacks.py:199-233) on the same bf16-rounded inputs and the same weights.

Tolerances are statistical: the HIP trunk rounds every activation to bf16 (relative
2^-9 per rounding, ~20 roundings deep) and runs its convolutions on bf16 weight
copies, so it differs from the fp32 oracle by accumulated rounding noise, not by a
reduction-order ulp.  Measured on MI355X (see each assertion) and bounded with a
~3x margin; a wrong formula or a dropped term shows up at O(1).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B, H = 64, 224


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30))


@pytest.fixture(scope="module")
def c2_run(dev):
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    from greedy_multimodal_learning_amd.engine import BalancedStep
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    from oracle import gating_ref, model_ref, weights
    g = torch.Generator().manual_seed(2024)
    # the bench's HBM layout: view-major channels_last bf16, exposed as [B, V, 3, H, W]
    buf = torch.randn(2, B, H, H, 3, generator=g).bfloat16()
    y = torch.randint(0, 40, (B,), generator=g)
    x_dev = buf.to(dev).permute(1, 0, 4, 2, 3)
    model = weights.apply_to_module(MMTM_MVCNN(), seed=5).to(dev)
    # locked gate (starting_epoch 2, epoch 1): d_BDR computed every step, no curation,
    # so every step sees the same forward; lr 0: parameters stay the oracle's
    gate = Bias_Mitigation_Strong(epsilon=0.01, curation_windowsize=5, branchnames=["net_view_0", "net_view_1"],
                                  starting_epoch=2)
    step = BalancedStep(model, lr=0.0, gate=gate, graphs=True)
    step.on_epoch_begin(1)
    yd = y.to(dev)
    losses = [float(step(x_dev, yd)) for _ in range(3)]  # eager, capture + replay, replay
    st = step.sync_gate()
    sums = step.norms.sums(grad_scale=1.0, lr=0.0).cpu().numpy()
    with torch.no_grad():
        mean, outs, _, _ = step.forward(x_dev)
    hip = dict(losses=losses, d_BDR=st["d_BDR"], sums=sums, mean=mean.float().cpu().numpy(),
               outs=[o.float().cpu().numpy() for o in outs], graphs=step.graphs, device_gate=step.device_gate)
    # oracle: fp32 on the CPU, same weights (seed 5), same bf16-rounded inputs
    torch.set_num_threads(max(1, min(32, torch.get_num_threads())))
    o = weights.apply_to_module(model_ref.MMTM_MVCNN_Ref(), seed=5)
    xo = buf.float().permute(1, 0, 4, 2, 3).contiguous()
    om, oo, _, _ = o(xo)
    oloss = gating_ref.blend_loss(oo, y)
    oloss.backward()
    osums = gating_ref.group_sums([(n, p, p.grad) for n, p in o.named_parameters()])
    od = gating_ref.BDRState(0.01, 5).update(osums)
    flat = [v for i in range(2) for v in (osums["wn_main"][i], osums["gn_main"][i])] + \
           [v for i in range(2) for v in (osums["wn_bypass"][i], osums["gn_bypass"][i])]
    ref = dict(loss=float(oloss.detach()), d_BDR=od, sums=np.asarray(flat, np.float64), mean=om.detach().numpy(),
               outs=[t.detach().numpy() for t in oo])
    # the bf16 floor: the same oracle under PyTorch's own CPU bf16 autocast (its convolutions
    # and matmuls in bf16, as the HIP trunk computes) against the fp32 oracle
    o16 = weights.apply_to_module(model_ref.MMTM_MVCNN_Ref(), seed=5)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        _, oo16, _, _ = o16(xo)
    gating_ref.blend_loss([t.float() for t in oo16], y).backward()
    s16 = gating_ref.group_sums([(n, p, p.grad) for n, p in o16.named_parameters()])
    od16 = gating_ref.BDRState(0.01, 5).update(s16)
    flat16 = [v for i in range(2) for v in (s16["wn_main"][i], s16["gn_main"][i])] + \
             [v for i in range(2) for v in (s16["wn_bypass"][i], s16["gn_bypass"][i])]
    ref["sums16"] = np.asarray(flat16, np.float64)
    ref["d_BDR16"] = od16
    return hip, ref


def test_c2_runs_the_benchmarked_configuration(c2_run):
    hip, _ = c2_run
    assert hip["graphs"] and hip["device_gate"]
    # lr 0 and a locked gate: the eager step, the captured step and the replay are one step
    assert hip["losses"][0] == pytest.approx(hip["losses"][1], rel=1e-6)
    assert hip["losses"][1] == hip["losses"][2]


def test_c2_logits_and_loss_vs_oracle(c2_run):
    hip, ref = c2_run
    e_mean = _rel(hip["mean"], ref["mean"])
    e_br = [_rel(a, b) for a, b in zip(hip["outs"], ref["outs"])]
    e_loss = abs(hip["losses"][-1] - ref["loss"]) / ref["loss"]
    print(f"C2 bf16 vs oracle: logits rel {e_mean:.3e} branches {e_br} loss rel {e_loss:.3e}")
    # measured: logits 1.07e-2 (branches 1.16e-2 / 0.97e-2), loss 4.1e-5
    assert e_mean < 3e-2 and max(e_br) < 3e-2
    assert e_loss < 2e-4
    # the predictions the accuracy metric reads: argmax agreement on all but near-ties
    agree = (hip["mean"].argmax(1) == ref["mean"].argmax(1)).mean()
    assert agree >= 0.9


def test_c2_group_sums_and_d_bdr_vs_oracle(c2_run):
    """The 8 per-branch sums compute_BDR takes (main0, main1, bypass0, bypass1: sum w^2,
    sum g^2) and d_BDR.  Weight sums are of the same fp32 masters: reduction order only.
    Gradient sums carry the trunk's bf16 noise; d_BDR = difference of log10 ratios."""
    hip, ref = c2_run
    w_h, w_r = hip["sums"][0::2], ref["sums"][0::2]
    g_h, g_r = hip["sums"][1::2], ref["sums"][1::2]
    e_w = np.abs(w_h - w_r) / w_r
    e_g = np.abs(g_h - g_r) / g_r
    e_d = abs(hip["d_BDR"] - ref["d_BDR"])
    f_g = np.abs(ref["sums16"][1::2] - g_r) / g_r  # PyTorch's own bf16 (CPU autocast) vs fp32
    f_d = abs(ref["d_BDR16"] - ref["d_BDR"])
    print(f"C2 bf16 vs oracle: weight sums rel {e_w.max():.3e}, grad sums rel {e_g}, "
          f"d_BDR {hip['d_BDR']:.6f} vs {ref['d_BDR']:.6f} (|diff| {e_d:.3e}); PyTorch CPU bf16 floor: "
          f"grad sums rel {f_g}, d_BDR |diff| {f_d:.3e}")
    # measured (round 3/4): weight sums 3.6e-8; gradient sums 7.9e-3 / 2.0e-4 / 8.0e-4 / 6.9e-4
    # (main0, main1, bypass0, bypass1) against a CPU bf16 floor of 7.8e-3 / 6.1e-3 / 6.5e-3 /
    # 6.0e-3 (B = 16, /tmp probe); which branch lands high follows the weights
    # (test_gpu_view_symmetry.py)
    assert e_w.max() < 1e-6
    # per branch within twice PyTorch's own bf16 error (a lucky small floor on one branch is
    # not held against it: half the largest floor is the least a branch is allowed)
    assert (e_g <= 2 * np.maximum(f_g, 0.5 * f_g.max()) + 1e-4).all(), (e_g, f_g)
    # d_BDR = sum of four log10 terms: no further from fp32 than the floor's worst case
    # (0.434 x the four gradient-sum errors of the bf16 floor); decision-level parity of the
    # same gate: test_gpu_gate_decisions.py, test_gpu_gate_steered.py
    assert e_d <= max(2 * f_d, 0.434 * f_g.sum()), (e_d, f_d, f_g)
