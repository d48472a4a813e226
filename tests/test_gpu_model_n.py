"""N-view models (configs C4 = 4 ResNet-18 modalities, C5 = 12 ResNet-50
views) against the oracle restatement `oracle.model_ref.MMTM_MVCNN_N_Ref` (N-way MMTM
of `oracle.mmtm_nway_ref`; the reference itself is 2-way ResNet-18 only, so N > 2 is
parity-unpinned w.r.t. the reference - at N = 2 the same code is pinned to the
reference's fixtures, tests/test_gpu_mmtm_n.py).

fp32 path (every trunk op on the HIP fp32 kernels): logits at rtol 1e-4 against the
oracle's fp32 CPU run; gradients within the envelope of that fp32 run's own error
against the oracle in float64 (the rule of tests/test_gpu_model.py)."""
import numpy as np
import pytest
import torch

from oracle import weights

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return np.abs(a - b) / np.maximum(np.abs(b), 1e-30)


def _oracle(trunk, V, x, y, dtype, caring=None):
    from oracle import gating_ref, model_ref
    o = weights.apply_to_module(model_ref.MMTM_MVCNN_N_Ref(num_views=V, trunk=trunk), seed=3).to(dtype)
    o.train(True)
    mean, outs, _, _ = o(x.to(dtype), curation_mode=caring is not None, caring_modality=caring)
    gating_ref.blend_loss(outs, y).backward()
    return o, mean.detach(), [u.detach() for u in outs]


@pytest.mark.parametrize("trunk,V,B,H,caring", [("resnet18", 4, 2, 64, None), ("resnet18", 4, 3, 64, 2),
                                                ("resnet50", 12, 2, 64, None)],
                         ids=["c4", "c4-curate2", "c5"])
def test_n_view_model_vs_oracle(trunk, V, B, H, caring):
    from greedy_multimodal_learning_amd.losses import blend_loss
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN_N
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(7)
    x = torch.randn(B, V, 3, H, H, generator=g)
    y = torch.randint(0, 40, (B,), generator=g)
    m = weights.apply_to_module(MMTM_MVCNN_N(num_views=V, trunk=trunk), seed=3).to(dev)
    m.train(True)
    mean, outs, _, _ = m(x.to(dev), curation_mode=caring is not None, caring_modality=caring)
    loss = blend_loss(outs, y.to(dev))
    loss.backward()
    o32, mean32, outs32 = _oracle(trunk, V, x, y, torch.float32, caring)
    o64, mean64, _ = _oracle(trunk, V, x, y, torch.float64, caring)
    assert [n for n, _ in m.named_parameters()] == [n for n, _ in o32.named_parameters()]
    np.testing.assert_allclose(mean.detach().cpu().numpy(), mean32.numpy(), rtol=1e-4, atol=1e-4)
    for u, v in zip(outs, outs32):
        np.testing.assert_allclose(u.detach().cpu().numpy(), v.numpy(), rtol=1e-4, atol=1e-4)
    # per-parameter gradient norms (what the N-branch gate reduces) vs float64
    g64 = dict(o64.named_parameters())
    g32 = dict(o32.named_parameters())
    names, e_ref, e_gpu = [], [], []
    for n, q in m.named_parameters():
        r = g64[n].grad
        if r is None:
            assert q.grad is None or float(q.grad.abs().max()) == 0.0, n  # curated modality's excitation
            continue
        n64 = float((r ** 2).sum())
        if n64 == 0:
            continue
        names.append(n)
        e_ref.append(abs(float((g32[n].grad.double() ** 2).sum()) - n64) / n64)
        e_gpu.append(abs(float((q.grad.double() ** 2).sum()) - n64) / n64)
    e_ref, e_gpu = np.array(e_ref), np.array(e_gpu)
    assert np.sqrt((e_gpu ** 2).mean()) <= max(3 * np.sqrt((e_ref ** 2).mean()), 2e-3), "grad-norm rms"
    assert e_gpu.max() <= max(10 * e_ref.max(), 1e-2), ("grad-norm max", names[int(e_gpu.argmax())])


@pytest.mark.parametrize("trunk,V,B", [("resnet18", 4, 8), ("resnet50", 12, 2)], ids=["c4", "c5"])
def test_engine_bf16_step_vs_oracle(trunk, V, B):
    """The benchmarked C4 / C5 steps (4 ResNet-18 / 12 ResNet-50 branches, bf16 trunk,
    hipGraphs, N-branch on-device gate) at 224x224: the step's loss, and the per-branch logits
    of the same model's bf16 forward, against the fp32 oracle on the same bf16-rounded
    inputs and weights (bf16 tolerance: 3e-2 of the loss / of the logit scale)."""
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    from greedy_multimodal_learning_amd.engine import BalancedStep
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN_N
    from oracle import gating_ref, model_ref
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(11)
    x = torch.randn(B, V, 3, 224, 224, generator=g).bfloat16()
    y = torch.randint(0, 40, (B,), generator=g)
    m = weights.apply_to_module(MMTM_MVCNN_N(num_views=V, trunk=trunk), seed=5)
    for p in m.parameters():  # the trunk computes on bf16 weights: start from bf16-exact ones
        p.data = p.data.bfloat16().float()
    o = model_ref.MMTM_MVCNN_N_Ref(num_views=V, trunk=trunk)
    missing, _ = o.load_state_dict(m.state_dict(), strict=False)
    assert not missing, missing
    o.train(True)
    _, outs_ref, _, _ = o(x.float())
    ref = float(gating_ref.blend_loss(outs_ref, y).detach())
    m = m.to(dev)
    xd, yd = x.to(dev), y.to(dev)
    m.train(True)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        _, outs, _, _ = m(xd)
    # the bf16 noise floor of this model and batch: the same oracle forward with its
    # convolutions in bf16 (CPU autocast), against the fp32 oracle
    o16 = model_ref.MMTM_MVCNN_N_Ref(num_views=V, trunk=trunk)
    o16.load_state_dict(m.state_dict(), strict=False)
    o16.train(True)
    with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
        _, outs16, _, _ = o16(x.float())
    for i, (u, u16, v) in enumerate(zip(outs, outs16, outs_ref)):
        u, u16, v = u.float().cpu(), u16.float(), v.detach()
        scale = float(v.abs().max()) + 1e-12
        err, floor = float((u - v).abs().max()) / scale, float((u16 - v).abs().max()) / scale
        assert err <= max(3e-2, 2 * floor), (f"branch {i} logits", err, "bf16 floor", floor)
    # epsilon 1e9: the gate computes every branch's BDR but never curates, so with lr 0
    # every step sees the same weights and the same MMTM path
    gate = Bias_Mitigation_Strong(epsilon=1e9, curation_windowsize=5, branchnames=m.branch_names(),
                                  starting_epoch=1, MMTMnames=m.mmtm_names())
    step = BalancedStep(m, lr=0.0, gate=gate, branchnames=m.branch_names(), MMTMnames=m.mmtm_names(),
                        graphs=True)
    step.on_epoch_begin(1)
    losses = [float(step(xd, yd)) for _ in range(3)]  # lr 0: every step sees the same weights
    assert losses[0] == losses[1] == losses[2] or max(losses) - min(losses) < 1e-3 * abs(ref)
    assert abs(losses[-1] - ref) <= 3e-2 * abs(ref), (losses, ref)
    assert step.device_gate and step.gate_n  # the N-branch on-device gate
    st = step.sync_gate()
    assert np.isfinite(gate.BDR).all() and len(gate.BDR) == V
    assert not st["curation_mode"] and st["n_curated"] == 0
