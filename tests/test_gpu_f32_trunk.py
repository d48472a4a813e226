"""Reference-precision (fp32) trunk kernels vs PyTorch in float64 on the CPU.

The fp32 path is what the reference's own loop drives (fp32 tensors, no autocast:
/root/reference/src/framework.py:146-148): convolutions on the exact-f32 MFMA
(gm_conv2d_f32), BatchNorm(+residual+ReLU) on the fp32 reduce/apply kernels
(gm_bn_*_f32), the stem max-pool (gm_maxpool2d_*_f32).  The only differences from
the fp64 values are fp32 rounding and summation order: tolerances are stated per
test (relative to the tensor's max), about 100x above the observed error and
1000x below a wrong formula.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
CL = torch.channels_last

SHAPES = [  # N, C, H, W, K, R, S, stride, pad
    (2, 3, 64, 64, 64, 7, 7, 2, 3),      # RGB stem, element-load path
    (1, 3, 37, 30, 64, 7, 7, 2, 3),      # stem, ragged
    (2, 64, 16, 16, 64, 3, 3, 1, 1),     # layer1
    (2, 64, 16, 16, 128, 3, 3, 2, 1),    # layer2 entry (strided dgrad)
    (2, 64, 16, 16, 128, 1, 1, 2, 0),    # downsample
    (3, 128, 9, 11, 256, 3, 3, 2, 1),    # ragged strided
    (2, 256, 4, 4, 512, 3, 3, 2, 1),
    (4, 512, 2, 2, 512, 3, 3, 1, 1),     # layer4 at 64x64 input
    (16, 64, 56, 56, 64, 3, 3, 1, 1),    # 128x128 tiles, long wgrad reduction (split)
    (2, 6, 7, 5, 12, 3, 3, 1, 1),        # C % 4 != 0: element path everywhere
    (1, 8, 5, 5, 20, 1, 1, 1, 0),
]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _err(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max()) / (float(b.abs().max()) + 1e-30)


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_conv_f32_fwd_dgrad_wgrad_vs_fp64(dev, shape):
    from greedy_multimodal_learning_amd.conv import GMConv2d
    N, C, H, W, K, R, S, st, pad = shape
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(K, C, R, S, generator=g) / (C * R * S) ** 0.5
    P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - S) // st + 1
    gy = torch.randn(N, K, P, Q, generator=g)
    xr, wr = x.double().requires_grad_(True), w.double().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=st, padding=pad)
    yr.backward(gy.double())
    m = GMConv2d(C, K, (R, S), stride=st, padding=pad, bias=False).to(dev)
    with torch.no_grad():
        m.weight.copy_(w)
    xd = x.to(dev).requires_grad_(True)  # NCHW in, like the reference's loader
    y = m(xd)
    assert y.dtype == torch.float32 and y.is_contiguous(memory_format=CL)
    assert "ConvF32" in type(y.grad_fn).__name__
    y.backward(gy.to(dev))
    assert _err(y, yr) < 2e-6
    assert _err(xd.grad, xr.grad) < 2e-6
    assert m.weight.grad.dtype == torch.float32
    assert _err(m.weight.grad, wr.grad) < 5e-6


def test_conv_f32_deterministic_accumulate_and_addend(dev):
    """Bit-identical reruns (split reductions summed in a fixed order); wgrad
    accumulate adds into the buffer; the dgrad addend (gradient join) is folded in."""
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import conv as G
    N, C, H, W, K, R, S, st, pad = 8, 64, 28, 28, 128, 3, 3, 2, 1
    gen = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(N, C, H, W, device=dev, generator=gen).contiguous(memory_format=CL)
    w = torch.randn(K, C, R, S, device=dev, generator=gen).contiguous(memory_format=CL)
    P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - S) // st + 1
    dy = torch.randn(N, K, P, Q, device=dev, generator=gen).contiguous(memory_format=CL)
    add = torch.randn(N, C, H, W, device=dev, generator=gen).contiguous(memory_format=CL)
    d = G._desc(N, H, W, C, K, R, S, st, pad)
    outs = []
    for _ in range(2):
        y = torch.empty(N, K, P, Q, device=dev).contiguous(memory_format=CL)
        dx = torch.empty(N, C, H, W, device=dev).contiguous(memory_format=CL)
        dxa = torch.empty_like(dx)
        dw = torch.empty(K, C, R, S, device=dev).contiguous(memory_format=CL)
        G.conv_f32(L.GM_CONV_FWD, d, x=x, w=w, out=y)
        G.conv_f32(L.GM_CONV_DGRAD, d, w=w, dy=dy, out=dx)
        G.conv_f32(L.GM_CONV_DGRAD, d, w=w, dy=dy, out=dxa, addend=add)
        G.conv_f32(L.GM_CONV_WGRAD, d, x=x, dy=dy, out=dw)
        outs.append((y, dx, dxa, dw.clone()))
        G.conv_f32(L.GM_CONV_WGRAD, d, x=x, dy=dy, out=dw, accumulate=True)
        torch.testing.assert_close(dw, 2 * outs[-1][3], rtol=1e-6, atol=1e-6)
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    torch.testing.assert_close(outs[0][2], outs[0][1] + add, rtol=1e-6, atol=1e-6)


BN_SHAPES = [(4, 64, 16, 16), (2, 128, 7, 7), (3, 8, 5, 5), (16, 512, 2, 2), (2, 2048, 4, 4), (16, 64, 56, 56)]


@pytest.mark.parametrize("shape", BN_SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("res,relu", [(False, False), (False, True), (True, True)])
def test_bn_f32_train_vs_fp64(dev, shape, res, relu):
    from greedy_multimodal_learning_amd.bn import GMBatchNorm2d
    N, C, H, W = shape
    g = torch.Generator().manual_seed(C + H)
    x = torch.randn(shape, generator=g) * 1.7 + 0.3
    r = torch.randn(shape, generator=g) if res else None
    w, b = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.1
    rm, rv = torch.randn(C, generator=g) * 0.1, torch.rand(C, generator=g) + 0.5
    dy = torch.randn(shape, generator=g)
    m = GMBatchNorm2d(C).to(dev)
    with torch.no_grad():
        m.weight.copy_(w); m.bias.copy_(b); m.running_mean.copy_(rm); m.running_var.copy_(rv)
    xg = x.to(dev).contiguous(memory_format=CL).requires_grad_(True)
    rg = r.to(dev).contiguous(memory_format=CL).requires_grad_(True) if res else None
    y = m(xg, residual=rg, relu=relu)
    assert y.dtype == torch.float32
    y.backward(dy.to(dev).contiguous(memory_format=CL))
    xr, wr, br = x.double().requires_grad_(True), w.double().requires_grad_(True), b.double().requires_grad_(True)
    rmr, rvr = rm.double(), rv.double()
    yr = F.batch_norm(xr, rmr, rvr, wr, br, training=True, momentum=0.1, eps=1e-5)
    rr = r.double().requires_grad_(True) if res else None
    if res:
        yr = yr + rr
    if relu:
        yr = F.relu(yr)
    yr.backward(dy.double())
    assert _err(y, yr) < 2e-6
    assert _err(xg.grad, xr.grad) < 5e-6
    assert _err(m.weight.grad, wr.grad) < 5e-6
    assert _err(m.bias.grad, br.grad) < 5e-6
    if res:
        assert _err(rg.grad, rr.grad) < 2e-6
    torch.testing.assert_close(m.running_mean.cpu().double(), rmr, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(m.running_var.cpu().double(), rvr, rtol=1e-6, atol=1e-7)
    assert int(m.num_batches_tracked) == 1
    m.eval()  # running statistics
    with torch.no_grad():
        ye = m(xg.detach(), residual=rg.detach() if res else None, relu=relu)
        yre = F.batch_norm(x.double(), rmr, rvr, w.double(), b.double(), training=False, eps=1e-5)
        if res:
            yre = yre + r.double()
        if relu:
            yre = F.relu(yre)
    assert _err(ye, yre) < 2e-6


@pytest.mark.parametrize("shape", [(2, 64, 32, 32), (3, 8, 9, 7), (1, 64, 112, 112)])
def test_maxpool_f32_exact(dev, shape):
    from greedy_multimodal_learning_amd.pool import GMMaxPool2d
    g = torch.Generator().manual_seed(shape[2])
    x = torch.randn(shape, generator=g)
    x[0, 0, :4, :4] = 0.5  # ties
    xg = x.to(dev).contiguous(memory_format=CL).requires_grad_(True)
    y = GMMaxPool2d(3, 2, 1)(xg)
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    gy = torch.randn(yr.shape, generator=g)
    y.backward(gy.to(dev).contiguous(memory_format=CL))
    yr.backward(gy)
    assert torch.equal(y.cpu(), yr)
    torch.testing.assert_close(xg.grad.cpu(), xr.grad, rtol=1e-6, atol=1e-6)


def test_resnet18_trunk_f32_vs_fp64(dev):
    """A whole ResNet-18 trunk (stem, 8 blocks, head) in fp32 on the HIP kernels vs the
    same weights in float64 (the oracle's torchvision-architecture restatement).
    Logits: 1e-4.  Gradients: a ReLU whose input lies within fp32 rounding of zero
    flips its mask in ANY fp32 run, and 20 layers amplify that (measured: the fp32 CPU
    oracle itself is off by up to 3e-2 on some parameters of this input), so the HIP
    gradients must stay inside the envelope of the fp32 CPU oracle's own error."""
    from greedy_multimodal_learning_amd.resnet import resnet18
    from oracle.resnet_ref import resnet18 as resnet18_ref
    torch.manual_seed(0)
    ref = resnet18_ref(num_classes=40).double()
    r32 = resnet18_ref(num_classes=40)
    r32.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    net = resnet18(num_classes=40)
    net.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    net = net.to(dev)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(4, 3, 64, 64, generator=g)
    out, o32, out_ref = net(x.to(dev)), r32(x), ref(x.double())
    assert _err(out, out_ref) < max(4 * _err(o32, out_ref), 1e-5)
    gy = torch.randn(out_ref.shape, generator=g)
    out.backward(gy.to(dev))
    o32.backward(gy)
    out_ref.backward(gy.double())
    rp, p32 = dict(ref.named_parameters()), dict(r32.named_parameters())
    e_hip = np.array([_err(p.grad, rp[n].grad) for n, p in net.named_parameters()])
    e_32 = np.array([_err(p32[n].grad, rp[n].grad) for n, _ in net.named_parameters()])
    assert np.sqrt((e_hip ** 2).mean()) <= max(3 * np.sqrt((e_32 ** 2).mean()), 1e-4), (e_hip, e_32)
    assert e_hip.max() <= max(10 * e_32.max(), 1e-4)
    assert np.median(e_hip) < 1e-2
