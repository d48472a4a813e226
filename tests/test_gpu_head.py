"""Fused classification heads (avgpool + fc of all branches) and the branch-summed
cross-entropy vs the PyTorch fp32 reference of the same ops (reference
src/model.py:53-56 head, train.py:22-29 blend_loss): values, every gradient,
in-place gradient delivery, a bad label."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last


def _rel(a, b):
    return (a.float() - b.float()).abs().max().item() / max(b.float().abs().max().item(), 1e-12)


@pytest.mark.parametrize("nb,B,C,H,N", [(2, 64, 512, 7, 40), (2, 5, 64, 3, 10), (3, 16, 128, 1, 7),
                                        (4, 33, 256, 4, 40), (2, 9, 64, 2, 130)])
def test_pooled_linear_and_xent_match_torch(nb, B, C, H, N):
    from greedy_multimodal_learning_amd.head import branch_xent, pooled_linear
    g = torch.Generator(device="cuda").manual_seed(B * C + H)
    fs = [torch.randn(B, C, H, H, device="cuda", generator=g).bfloat16().contiguous(memory_format=CL)
          for _ in range(nb)]
    fcs = [nn.Linear(C, N).cuda() for _ in range(nb)]
    y = torch.randint(0, N, (B,), device="cuda", generator=g)
    fh = [f.clone().requires_grad_(True) for f in fs]
    outs = pooled_linear(fh, fcs)
    loss = branch_xent(outs, y)
    loss.backward()
    fr = [f.float().requires_grad_(True) for f in fs]
    ws = [fc.weight.detach().clone().requires_grad_(True) for fc in fcs]
    bs = [fc.bias.detach().clone().requires_grad_(True) for fc in fcs]
    refs = [F.linear(torch.flatten(F.adaptive_avg_pool2d(f, 1), 1), w, b) for f, w, b in zip(fr, ws, bs)]
    lr = sum(F.cross_entropy(o, y) for o in refs)
    lr.backward()
    for o, r in zip(outs, refs):
        assert o.dtype == torch.float32 and o.shape == (B, N)
        assert _rel(o, r) < 1e-5
    assert abs(loss.item() - lr.item()) <= 1e-5 * abs(lr.item())
    for i in range(nb):
        assert _rel(fcs[i].weight.grad, ws[i].grad) < 1e-5
        assert _rel(fcs[i].bias.grad, bs[i].grad) < 1e-5
        assert fh[i].grad.dtype == torch.bfloat16 and fh[i].grad.is_contiguous(memory_format=CL)
        assert _rel(fh[i].grad, fr[i].grad) < 1e-2  # bf16 activation gradient


def test_xent_separate_tensors_and_scaled_grad():
    from greedy_multimodal_learning_amd.head import branch_xent
    g = torch.Generator(device="cuda").manual_seed(1)
    xs = [torch.randn(8, 5, device="cuda", generator=g).requires_grad_(True) for _ in range(2)]
    y = torch.tensor([0, 1, 2, 3, 4, 0, 1, 2], device="cuda")
    (3.0 * branch_xent(xs, y)).backward()
    xr = [x.detach().clone().requires_grad_(True) for x in xs]
    (3.0 * sum(F.cross_entropy(x, y) for x in xr)).backward()
    for a, b in zip(xs, xr):
        torch.testing.assert_close(a.grad, b.grad, rtol=1e-5, atol=1e-6)


def test_xent_bad_label_is_nan():
    from greedy_multimodal_learning_amd.head import branch_xent
    x = torch.randn(4, 3, device="cuda")
    assert torch.isnan(branch_xent([x], torch.tensor([0, 1, 3, 2], device="cuda")))


def test_head_grad_sink_in_place():
    """Engine mode: fc weight/bias gradients land in .grad in place (overwrite stale
    content on first use) and the sink's hook fires once per parameter."""
    from greedy_multimodal_learning_amd.gradsink import GradSink
    from greedy_multimodal_learning_amd.head import branch_xent, pooled_linear
    fs = [torch.randn(8, 64, 2, 2, device="cuda").bfloat16().contiguous(memory_format=CL) for _ in range(2)]
    fcs = [nn.Linear(64, 10).cuda() for _ in range(2)]
    y = torch.randint(0, 10, (8,), device="cuda")
    branch_xent(pooled_linear(fs, fcs), y).backward()
    ref = [p.grad.clone() for fc in fcs for p in fc.parameters()]
    for fc in fcs:
        for p in fc.parameters():
            p.grad.fill_(5.0)
    fired = []
    sink = GradSink([p for fc in fcs for p in fc.parameters()], on_ready=fired.append)
    sink.begin_step()
    branch_xent(pooled_linear(fs, fcs), y).backward()
    sink.end_step()
    sink.detach()
    assert len(fired) == 4
    for r, p in zip(ref, [p for fc in fcs for p in fc.parameters()]):
        assert torch.equal(r, p.grad)
