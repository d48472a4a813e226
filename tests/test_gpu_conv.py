"""bf16 MFMA implicit-GEMM convolutions (fwd / dgrad / wgrad) vs PyTorch fp32 on the CPU.

Inputs and weights are rounded to bf16 first, so every product is exact in fp32 and
the only differences are fp32 summation order and the bf16 rounding of the
activation outputs (fwd, dgrad: 2^-8 relative) -> tolerance 1e-2 of the tensor's
max; the fp32 weight gradient -> 2e-3 of its max.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

WGRAD_LOOP_DEFAULT = 22  # gm_conv_set_wgrad_loop's default (conv_wgrad.hip g_wgrad_loop)

SHAPES = [  # N, C, H, W, K, R, S, stride, pad
    (2, 64, 56, 56, 64, 3, 3, 1, 1),
    (2, 64, 56, 56, 128, 3, 3, 2, 1),
    (2, 64, 56, 56, 128, 1, 1, 2, 0),
    (2, 128, 28, 28, 128, 3, 3, 1, 1),
    (2, 256, 14, 14, 512, 3, 3, 2, 1),
    (2, 512, 7, 7, 512, 3, 3, 1, 1),
    (2, 3, 64, 64, 64, 7, 7, 2, 3),
    (3, 64, 9, 11, 64, 3, 3, 2, 1),
    (1, 8, 5, 5, 16, 3, 3, 1, 1),
    (5, 128, 7, 7, 256, 1, 1, 2, 0),
]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _close(a, b, tol):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    scale = float(b.abs().max()) + 1e-12
    np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=0, atol=tol * scale)


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_conv_fwd_dgrad_wgrad(dev, shape):
    from greedy_multimodal_learning_amd.conv import GMConv2d
    N, C, H, W, K, R, S, st, pad = shape
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(N, C, H, W, generator=g).bfloat16()
    w = (torch.randn(K, C, R, S, generator=g) / (C * R * S) ** 0.5).bfloat16()
    gy_shape = (N, K, (H + 2 * pad - R) // st + 1, (W + 2 * pad - S) // st + 1)
    gy = torch.randn(*gy_shape, generator=g).bfloat16()
    # reference: fp32 on the CPU from the bf16-rounded values
    xr, wr = x.float().requires_grad_(True), w.float().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=st, padding=pad)
    yr.backward(gy.float())
    # HIP
    m = GMConv2d(C, K, (R, S), stride=st, padding=pad, bias=False).to(dev)
    with torch.no_grad():
        m.weight.copy_(w.float())
    m = m.to(memory_format=torch.channels_last)
    xd = x.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = m(xd)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    y.backward(gy.to(dev).contiguous(memory_format=torch.channels_last))
    _close(y, yr, 1e-2)
    _close(xd.grad, xr.grad, 1e-2)
    assert m.weight.grad.dtype == torch.float32
    _close(m.weight.grad, wr.grad, 2e-3)


def test_conv_fp32_input_runs_hip_f32(dev):
    """fp32 inputs take the exact-f32 MFMA kernels (gm_conv2d_f32), not a vendor library."""
    from greedy_multimodal_learning_amd.conv import GMConv2d
    m = GMConv2d(8, 8, 3, padding=1, bias=False).to(dev)
    x = torch.randn(1, 8, 5, 5, device=dev)
    y = m(x)
    assert y.dtype == torch.float32 and "ConvF32" in type(y.grad_fn).__name__ if y.grad_fn else True
    torch.testing.assert_close(y, F.conv2d(x, m.weight, padding=1), rtol=1e-5, atol=1e-5)


def test_conv_wgrad_in_place_sink(dev):
    """Engine mode: the weight gradient is written into .grad in place (first use
    overwrites stale content, second use in the same step accumulates)."""
    from greedy_multimodal_learning_amd.conv import GMConv2d
    from greedy_multimodal_learning_amd.gradsink import GradSink
    CL = torch.channels_last
    m = GMConv2d(64, 64, 3, padding=1, bias=False).to(dev).to(memory_format=CL)
    x = torch.randn(2, 64, 14, 14, device=dev).bfloat16().contiguous(memory_format=CL)
    gy = torch.randn(2, 64, 14, 14, device=dev).bfloat16().contiguous(memory_format=CL)
    m(x).backward(gy)
    ref = m.weight.grad.clone()
    m.weight.grad = torch.full_like(ref, 3.0).contiguous(memory_format=CL)
    fired = []
    sink = GradSink([m.weight], on_ready=fired.append)
    sink.begin_step()
    m(x).backward(gy)
    first = m.weight.grad.clone()
    m(x).backward(gy)
    sink.end_step()
    sink.detach()
    assert len(fired) == 2
    assert torch.equal(first, ref)
    torch.testing.assert_close(m.weight.grad, 2 * ref, rtol=1e-6, atol=1e-6)


def test_weight_prep_multi_matches_single(dev):
    """One-launch multi-tensor weight prep == the per-convolution prep, bit for bit
    (bf16 KRSC copy with zero-padded channels + transposed dgrad copy)."""
    from greedy_multimodal_learning_amd.conv import GMConv2d, WeightPrep, _cpad, weight_prep
    CL = torch.channels_last
    torch.manual_seed(3)
    net = torch.nn.Sequential(GMConv2d(3, 64, 7, stride=2, padding=3, bias=False),
                              GMConv2d(64, 128, 3, padding=1, bias=False),
                              GMConv2d(128, 256, 1, stride=2, bias=False),
                              GMConv2d(256, 72, 3, padding=1, bias=False),
                              GMConv2d(72, 70, 1, bias=False)).to(dev).to(memory_format=CL)
    # (ragged tiles: K 72 and 70 - element-wise transposed stores -, C 3 - element-wise loads)
    assert net[0].uses_pair_stem() and len(WeightPrep(net).copies) == 4  # the pair-view stem packs its own
    net[0].pair_stem = False
    wp = WeightPrep(net)
    wp.run()
    torch.cuda.synchronize()
    for (w, wb, wt), m in zip(wp.copies, net):
        rb, rt = weight_prep(m.weight, _cpad(m.weight.shape[1]), wt is not None)
        assert torch.equal(wb, rb)
        if wt is not None:
            assert torch.equal(wt, rt)
    assert wp.copies[0][2] is None  # stem: no transposed copy


@pytest.mark.parametrize("shape", [(2, 3, 64, 64, 64, 7, 7, 2, 3), (1, 3, 224, 224, 64, 7, 7, 2, 3),
                                   (3, 3, 37, 30, 64, 7, 7, 2, 3), (2, 4, 16, 18, 32, 5, 5, 2, 2)],
                         ids=lambda s: "x".join(map(str, s)))
def test_stem_pixel_pair_path(dev, shape):
    """The RGB stem on the zero-bordered pixel-pair view (strides (2,1), K = R*ceil(S/2)*8)
    == the fp32 convolution; weight gradient delivered in the parameter's layout."""
    from greedy_multimodal_learning_amd.conv import GMConv2d
    N, C, H, W, K, R, S, st, pad = shape
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(N, C, H, W, generator=g).bfloat16()
    w = (torch.randn(K, C, R, S, generator=g) / (C * R * S) ** 0.5).bfloat16()
    gy_shape = (N, K, (H + 2 * pad - R) // st + 1, (W + 2 * pad - S) // st + 1)
    gy = torch.randn(*gy_shape, generator=g).bfloat16()
    wr = w.float().requires_grad_(True)
    yr = F.conv2d(x.float(), wr, stride=st, padding=pad)
    yr.backward(gy.float())
    m = GMConv2d(C, K, (R, S), stride=st, padding=pad, bias=False).to(dev)
    with torch.no_grad():
        m.weight.copy_(w.float())
    m = m.to(memory_format=torch.channels_last)
    assert m.uses_pair_stem()
    xd = x.to(dev).contiguous(memory_format=torch.channels_last)
    y = m(xd)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    assert y.grad_fn is not None and "Stem" in type(y.grad_fn).__name__
    y.backward(gy.to(dev).contiguous(memory_format=torch.channels_last))
    _close(y, yr, 1e-2)
    _close(m.weight.grad, wr.grad, 2e-3)


@pytest.mark.parametrize("shape", [(64, 256, 14, 14, 256, 3, 3, 1, 1), (64, 512, 7, 7, 512, 3, 3, 1, 1),
                                   (64, 256, 14, 14, 512, 3, 3, 2, 1), (8, 512, 7, 7, 512, 3, 3, 1, 1), (64, 256, 14, 14, 512, 3, 3, 2, 1)],
                         ids=lambda s: "x".join(map(str, s)))
def test_conv_splitk_turnstile(dev, shape):
    """Layer-3/4 shapes take 128x128 tiles with K split over 2-4 workgroups that hand
    their fp32 accumulators on in a fixed order: same result as the fp32 convolution,
    bit-identical across runs (deterministic), workspace left reusable."""
    import ctypes
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import conv as G
    N, C, H, W, K, R, S, st, pad = shape
    d = G._desc(N, H, W, C, K, R, S, st, pad)
    assert L.load().gm_conv2d_splitk_ws_bytes(ctypes.byref(d), 0) > 0  # the split path is taken
    g = torch.Generator(device="cuda").manual_seed(sum(shape))
    CL = torch.channels_last
    x = torch.randn(N, C, H, W, device=dev, generator=g).bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(K, C, R, S, device=dev, generator=g) / (C * R * S) ** 0.5).bfloat16().contiguous(memory_format=CL)
    P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - S) // st + 1
    dy = torch.randn(N, K, P, Q, device=dev, generator=g).bfloat16().contiguous(memory_format=CL)
    y1, y2 = G.conv_fwd(x, w, st, pad), G.conv_fwd(x, w, st, pad)
    dx1, dx2 = G.conv_dgrad(dy, w, H, W, st, pad), G.conv_dgrad(dy, w, H, W, st, pad)
    assert torch.equal(y1, y2) and torch.equal(dx1, dx2)
    yr = F.conv2d(x.float(), w.float(), stride=st, padding=pad)
    dxr = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [st, st], [pad, pad], [1, 1],
                                              False, [0, 0], 1, [True, False, False])[0]
    _close(y1, yr, 1e-2)
    _close(dx1, dxr, 1e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(3, 2, 3, 37, 30, 64, 7, 7, 3), (2, 2, 3, 224, 224, 64, 7, 7, 3),
                                   (2, 1, 4, 16, 18, 32, 5, 5, 2), (1, 3, 1, 9, 9, 8, 3, 3, 1)],
                         ids=lambda s: "x".join(map(str, s)))
def test_stem_pack_kernel_matches_torch_pack(dev, shape, dtype):
    """gm_stem_pack_bf16 (input + weight pair views, one launch) == the PyTorch packing,
    bit for bit, from a strided view of a [B, V, C, H, W] batch."""
    from greedy_multimodal_learning_amd import conv as G
    N, V, C, H, W, K, R, S, pad = shape
    g = torch.Generator(device="cuda").manual_seed(sum(shape))
    batch = torch.randn(N, V, C, H, W, device=dev, generator=g).to(dtype)
    w = torch.randn(K, C, R, S, device=dev, generator=g)
    x = batch[:, V - 1]
    xp, wp = G.stem_pack(x, w, pad)
    assert torch.equal(xp, G.stem_pack_input(x, R, S, pad))
    assert torch.equal(wp, G.stem_pack_weight(w))
    # the model's channels_last weight parameter, read at its strides (no contiguous copy)
    _, wp_cl = G.stem_pack(x, w.contiguous(memory_format=torch.channels_last), pad)
    assert torch.equal(wp_cl, wp)


def test_conv_splitk_spin_timeout_never_silent(dev):
    """A split that runs out of its poll budget (forced: 1 poll) must not add a stale
    running sum: either every split saw its predecessor in time (exact result, no
    fault) or the fault word is raised and the affected outputs are NaN.  After the
    fault check repairs the workspaces, the default budget gives exact results again."""
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import conv as G
    lib = L.load()
    L.device_faults(clear=True)
    N, C, H, W, K, R, S, st, pad = 64, 512, 7, 7, 512, 3, 3, 1, 1
    g = torch.Generator(device="cuda").manual_seed(9)
    CL = torch.channels_last
    x = torch.randn(N, C, H, W, device=dev, generator=g).bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(K, C, R, S, device=dev, generator=g) / (C * R * S) ** 0.5).bfloat16().contiguous(memory_format=CL)
    ref = G.conv_fwd(x, w, st, pad)
    try:
        L.check(lib.gm_set_spin_limit(1), "gm_set_spin_limit")
        ys = [G.conv_fwd(x, w, st, pad) for _ in range(4)]
        torch.cuda.synchronize()
    finally:
        lib.gm_set_spin_limit(0)
    faults = L.device_faults()
    if faults & L.GM_FAULT_SPLITK_SPIN:
        assert any(torch.isnan(y.float()).any() for y in ys)
        with pytest.raises(L.GreedyMMLError, match="split-K"):
            L.check_device_faults()
    else:
        assert all(torch.equal(y, ref) for y in ys)
    assert L.device_faults() == 0
    assert torch.equal(G.conv_fwd(x, w, st, pad), ref)


@pytest.mark.parametrize("shape", [(4, 128, 28, 28, 128, 3, 3, 1, 1), (4, 64, 56, 56, 128, 3, 3, 2, 1),
                                   (64, 256, 14, 14, 256, 3, 3, 1, 1), (5, 128, 7, 7, 256, 1, 1, 2, 0),
                                   (4, 64, 56, 56, 64, 3, 3, 1, 1)],
                         ids=lambda s: "x".join(map(str, s)))
def test_conv_dgrad_fused_addend(dev, shape):
    """The input-gradient epilogue's fused gradient join (dx = dgrad + addend, the
    residual branch's gradient) on the halo, im2col, split-K and layer-1 resident-weight
    kernels (every identity block joins in place, layer 1 included): equal to the fp32
    reference plus the addend, and to the unfused dgrad plus the addend."""
    from greedy_multimodal_learning_amd import conv as G
    N, C, H, W, K, R, S, st, pad = shape
    g = torch.Generator(device="cuda").manual_seed(sum(shape) + 1)
    CL = torch.channels_last
    x = torch.randn(N, C, H, W, device=dev, generator=g).bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(K, C, R, S, device=dev, generator=g) / (C * R * S) ** 0.5).bfloat16().contiguous(memory_format=CL)
    P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - S) // st + 1
    dy = torch.randn(N, K, P, Q, device=dev, generator=g).bfloat16().contiguous(memory_format=CL)
    add = torch.randn(N, C, H, W, device=dev, generator=g).bfloat16().contiguous(memory_format=CL)
    wt = w.permute(1, 0, 2, 3).contiguous(memory_format=CL)
    dx = G.conv_dgrad_t(dy, wt, H, W, st, pad)
    dxa = G.conv_dgrad_t(dy, wt, H, W, st, pad, addend=add)
    dxr = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [st, st], [pad, pad], [1, 1],
                                              False, [0, 0], 1, [True, False, False])[0]
    _close(dxa, dxr + add.float(), 1e-2)
    _close(dxa, dx.float() + add.float(), 1e-2)
    # in place over the addend (the gradient join's pending tensor): bit-identical
    buf = add.clone()
    dxi = G.conv_dgrad_t(dy, wt, H, W, st, pad, addend=buf, inplace=True)
    assert dxi.data_ptr() == buf.data_ptr()
    assert torch.equal(dxi, dxa)


@pytest.mark.parametrize("shape", [(64, 2, 224, 224), (8, 1, 224, 224), (3, 2, 64, 64), (2, 1, 96, 72),
                                   (300, 1, 40, 38)],
                         ids=lambda s: "x".join(map(str, s)))
def test_stem_wgrad_kernel(dev, shape):
    """The pixel-pair stem's weight gradient on k_wgrad_stem (one wave per tap row,
    per-workgroup fp32 partials + the fixed-order split sum), G view groups in one launch,
    equals k_conv_wgrad4 (same bf16 operands, fp32 sums in another order) and the fp32
    weight gradient of the pair-view convolution; bit-identical on a second run."""
    import ctypes
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import conv as CV
    lib = L.load()
    B, G, H, W = shape
    K, R = 64, 7
    P, Q, Sp, Hp, Wp = CV._stem_geom(H, W, R, R, 3)
    g = torch.Generator(device="cuda").manual_seed(sum(shape))
    xp = torch.empty(G * B, Hp, Wp // 2, 8, device=dev, dtype=torch.bfloat16)
    for v in range(G):
        x = torch.randn(B, 3, H, W, device=dev, generator=g)
        CV.stem_pack(x, torch.randn(K, 3, R, R, device=dev, generator=g), 3, xp=xp[v * B:(v + 1) * B],
                     wp=torch.empty(K, R, Sp, 8, device=dev, dtype=torch.bfloat16))
    dy = torch.randn(G * B, P, Q, K, device=dev, generator=g).bfloat16()
    d = CV._desc_hw(B, Hp, Wp // 2, 8, K, R, Sp, 2, 1, 0, 0)
    n = K * R * Sp * 8

    def run(on):
        L.check(lib.gm_conv_set_wgrad_stem(on), "gm_conv_set_wgrad_stem")
        need = lib.gm_conv2d_wgrad_grouped_scratch(ctypes.byref(d), G)
        scr = torch.empty(max(need, 16), device=dev, dtype=torch.uint8)
        dw = torch.full((G, K, R, Sp, 8), float("nan"), device=dev)
        L.check(lib.gm_conv2d_wgrad_grouped_bf16(ctypes.byref(d), G, dy.data_ptr(), xp.data_ptr(), dw.data_ptr(), n, 8,
                                                 0, scr.data_ptr(), need, L.stream_of(dev)), "wgrad")
        torch.cuda.synchronize()
        return dw
    try:
        d_new, d_new2, d_old = run(1), run(1), run(0)
    finally:
        lib.gm_conv_set_wgrad_stem(1)
    assert torch.isfinite(d_new).all()
    assert torch.equal(d_new, d_new2)
    _close(d_new, d_old, 1e-5)
    for v in range(G):  # fp32 reference on the pair view: [B, 8, Hp, Wp/2] x [64, 8, 7, 4], strides (2, 1)
        xv = xp[v * B:(v + 1) * B].permute(0, 3, 1, 2).float()
        dyv = dy[v * B:(v + 1) * B].permute(0, 3, 1, 2).float()
        ref = torch.nn.grad.conv2d_weight(xv, (K, 8, R, Sp), dyv, stride=(2, 1))
        _close(d_new[v].permute(0, 3, 1, 2), ref, 1e-5)


@pytest.mark.parametrize("shape", [(64, 3, 224, 224), (3, 3, 37, 30), (2, 3, 64, 64), (5, 3, 250, 200),
                                   (300, 3, 40, 36), (1, 3, 224, 224)],
                         ids=lambda s: "x".join(map(str, s)))
def test_stem_resident_weight_kernel(dev, shape):
    """The pixel-pair stem (7x7/s2, 3 -> 64 channels) on the resident-weight kernel
    (weights in LDS, a workgroup per run of output rows, input rows streamed through an LDS
    ring) equals the im2col kernel and the fp32 convolution: one chunk per image (N = 300),
    one row per chunk (N = 1), ragged last chunks (P = 125, 19)."""
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import conv as G
    lib = L.load()
    N, C, H, W = shape
    g = torch.Generator(device="cuda").manual_seed(sum(shape))
    x = torch.randn(N, C, H, W, device=dev, generator=g)
    w = torch.randn(64, C, 7, 7, device=dev, generator=g) / (C * 49) ** 0.5
    P, Q, Sp, Hp, Wp = G._stem_geom(H, W, 7, 7, 3)
    xp, wp = G.stem_pack(x, w, 3)
    try:
        L.check(lib.gm_conv_set_stem(0), "gm_conv_set_stem")
        y0 = G.stem_fwd(xp, wp, P, Q)
        L.check(lib.gm_conv_set_stem(1), "gm_conv_set_stem")
        y1 = G.stem_fwd(xp, wp, P, Q)
        torch.cuda.synchronize()
    finally:
        lib.gm_conv_set_stem(1)
    yr = F.conv2d(x.bfloat16().float(), w.bfloat16().float(), stride=2, padding=3)
    _close(y1, yr, 1e-2)
    _close(y1, y0, 1e-2)


HALO_SHAPES = [  # N, C, H, W, K: 3x3 / stride 1 / pad 1 (ResNet layers 2-4 and a ragged batch)
    (8, 128, 28, 28, 128),   # 256-pixel tiles unsplit
    (8, 256, 14, 14, 256),   # split-K 2 through the turnstile
    (8, 512, 7, 7, 512),     # split-K 4
    (3, 128, 9, 11, 256),    # tiles spanning images, a partial last tile
]


@pytest.mark.parametrize("mode", [1, 2], ids=["halo128", "halo256"])
@pytest.mark.parametrize("shape", HALO_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_conv_halo_tiles(dev, shape, mode):
    """The halo-staged kernel in its 128- and 256-pixel tile forms (gm_conv_set_halo 1 / 2)
    vs fp32 PyTorch: forward and the stride-1 input gradient."""
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import conv as G
    N, C, H, W, K = shape
    g = torch.Generator().manual_seed(sum(shape) + mode)
    x = torch.randn(N, C, H, W, generator=g).bfloat16()
    w = (torch.randn(K, C, 3, 3, generator=g) / (C * 9) ** 0.5).bfloat16()
    gy = torch.randn(N, K, H, W, generator=g).bfloat16()
    xr, wr = x.float().requires_grad_(True), w.float()
    yr = F.conv2d(xr, wr, padding=1)
    yr.backward(gy.float())
    cl = torch.channels_last
    lib = L.load()
    L.check(lib.gm_conv_set_halo(mode), "gm_conv_set_halo")
    try:
        xd, wd = x.to(dev).contiguous(memory_format=cl), w.to(dev).contiguous(memory_format=cl)
        y = G.conv_fwd(xd, wd, 1, 1)
        wt = wd.permute(1, 0, 2, 3).contiguous(memory_format=cl)
        dx = G.conv_dgrad_t(gy.to(dev).contiguous(memory_format=cl), wt, H, W, 1, 1)
        torch.cuda.synchronize()
        assert L.device_faults(clear=True) == 0
    finally:
        lib.gm_conv_set_halo(1)
    _close(y, yr, 1e-2)
    _close(dx, xr.grad, 1e-2)


@pytest.mark.parametrize("shape", [SHAPES[0], SHAPES[1], SHAPES[2], SHAPES[4], SHAPES[6], SHAPES[8]],
                         ids=lambda s: "x".join(map(str, s)))
def test_wgrad_staging_forms_bit_identical(dev, shape):
    """k_conv_wgrad4's register-staged operands and LDS-DMA staging build the same LDS
    image and run the same MFMAs: bit-identical weight gradients."""
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd.conv import GMConv2d
    N, C, H, W, K, R, S, st, pad = shape
    CL = torch.channels_last
    torch.manual_seed(sum(shape))
    m = GMConv2d(C, K, (R, S), stride=st, padding=pad, bias=False).to(dev).to(memory_format=CL)
    x = torch.randn(N, C, H, W, device=dev).bfloat16().contiguous(memory_format=CL)
    gy_shape = (N, K, (H + 2 * pad - R) // st + 1, (W + 2 * pad - S) // st + 1)
    gy = torch.randn(*gy_shape, device=dev).bfloat16().contiguous(memory_format=CL)
    lib = L.load()
    grads = []
    try:
        for wr in (1, 0):
            L.check(lib.gm_conv_set_wgrad_staging(wr), "wgrad staging")
            m.weight.grad = None
            m(x).backward(gy)
            grads.append(m.weight.grad.clone())
    finally:
        L.check(lib.gm_conv_set_wgrad_staging(2), "wgrad staging")  # the default
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("shape", [(8, 64, 56, 56, 64, 3, 1, 1), (3, 64, 56, 56, 128, 3, 2, 1),
                                   (8, 128, 28, 28, 128, 3, 1, 1), (5, 256, 14, 14, 256, 3, 1, 1),
                                   (64, 512, 7, 7, 512, 3, 1, 1), (7, 256, 14, 14, 512, 1, 2, 0),
                                   (2, 8, 115, 115, 64, 7, 1, 0)],
                         ids=lambda s: "x".join(map(str, s)))
def test_wgrad4_grouped_vs_fp32(dev, shape):
    """k_conv_wgrad4 (the im2col weight gradient every shape can take; the halo kernel off so
    the 3x3 / s1 shapes take it too) grouped over two views, split-K and ragged tails included
    (B = 3, 5, 7), plain and accumulating, against fp32 PyTorch per group."""
    import ctypes
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import conv as CV
    N, C, H, W, K, R, st, pad = shape
    G = 2
    P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
    torch.manual_seed(sum(shape))
    x = torch.randn(G * N, H, W, C, device=dev).bfloat16()
    dy = torch.randn(G * N, P, Q, K, device=dev).bfloat16()
    lib = L.load()
    d = CV._desc_hw(N, H, W, C, K, R, R, st, st, pad, pad)
    outs = []
    try:
        L.check(lib.gm_conv_set_wgrad_loop(0), "loop")
        need = lib.gm_conv2d_wgrad_grouped_scratch(ctypes.byref(d), G)
        scr = torch.empty(max(need, 16), device=dev, dtype=torch.uint8)
        for acc in (0, 1):
            dw = torch.full((G, K, R, R, C), 0.25, device=dev, dtype=torch.float32)
            L.check(lib.gm_conv2d_wgrad_grouped_bf16(ctypes.byref(d), G, dy.data_ptr(), x.data_ptr(),
                                                      dw.data_ptr(), K * R * R * C, C, acc, scr.data_ptr(),
                                                      need, L.stream_of(dev)), "wgrad")
            outs.append(dw)
        torch.cuda.synchronize()
    finally:
        L.check(lib.gm_conv_set_wgrad_loop(WGRAD_LOOP_DEFAULT), "loop")  # the default
    for gi in range(G):
        xr = x[gi * N:(gi + 1) * N].float().permute(0, 3, 1, 2)
        gr = dy[gi * N:(gi + 1) * N].float().permute(0, 3, 1, 2)
        ref = torch.nn.grad.conv2d_weight(xr, (K, C, R, R), gr, stride=st, padding=pad)
        for acc, base in ((0, 0.0), (1, 0.25)):
            got = outs[acc][gi].permute(0, 3, 1, 2) - base
            err = float((got - ref).abs().max() / ref.abs().max())
            assert err < 2e-3, (gi, acc, err)


@pytest.mark.parametrize("shape", [(64, 56, 56, 64), (3, 56, 56, 64), (5, 20, 20, 64), (2, 9, 7, 64), (1, 3, 62, 64),
                                   (64, 28, 28, 128), (3, 28, 28, 128), (2, 5, 9, 128), (3, 30, 30, 128),
                                   (64, 14, 14, 256), (3, 14, 14, 256), (2, 6, 13, 128), (64, 7, 7, 512),
                                   (3, 7, 7, 512), (1, 4, 14, 256), (2, 5, 9, 256)],
                         ids=lambda s: "x".join(map(str, s)))
def test_wgrad_halo64_vs_fp32(dev, shape):
    """k_wgrad_halo64 (3x3 / s1 weight gradient: 64 x 9 x 64 gradient blocks in one workgroup's
    accumulators, super-rows of 64 / PP image rows staged once for all nine taps, rows split
    over the workgroups, slabs summed in a fixed order; PP = 64, 32, 16 for layers 1, 2, 3-4)
    against fp32 PyTorch, grouped over two views, plain and accumulating, ragged batches and
    image heights that straddle super-rows included; and against k_conv_wgrad4 within fp32
    summation-order noise."""
    import ctypes
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import conv as CV
    N, H, W, C = shape
    K = C
    G = 2
    mode = 2 if C == 64 else (6 if C == 128 else 14)
    torch.manual_seed(N * 1000 + H * 10 + W)
    x = torch.randn(G * N, H, W, C, device=dev).bfloat16()
    dy = torch.randn(G * N, H, W, K, device=dev).bfloat16()
    lib = L.load()
    d = CV._desc_hw(N, H, W, C, K, 3, 3, 1, 1, 1, 1)
    outs = {}
    try:
        for m in (0, mode):
            L.check(lib.gm_conv_set_wgrad_loop(m), "loop")
            need = lib.gm_conv2d_wgrad_grouped_scratch(ctypes.byref(d), G)
            scr = torch.empty(max(need, 16), device=dev, dtype=torch.uint8)
            res = []
            for acc in (0, 1):
                dw = torch.full((G, K, 3, 3, C), 0.5, device=dev, dtype=torch.float32)
                L.check(lib.gm_conv2d_wgrad_grouped_bf16(ctypes.byref(d), G, dy.data_ptr(), x.data_ptr(),
                                                          dw.data_ptr(), K * 9 * C, C, acc, scr.data_ptr(),
                                                          need, L.stream_of(dev)), "wgrad")
                res.append(dw)
            outs[m] = res
        torch.cuda.synchronize()
    finally:
        L.check(lib.gm_conv_set_wgrad_loop(WGRAD_LOOP_DEFAULT), "loop")  # the default
    for gi in range(G):
        xr = x[gi * N:(gi + 1) * N].float().permute(0, 3, 1, 2)
        gr = dy[gi * N:(gi + 1) * N].float().permute(0, 3, 1, 2)
        ref = torch.nn.grad.conv2d_weight(xr, (K, C, 3, 3), gr, stride=1, padding=1)
        for acc, base in ((0, 0.0), (1, 0.5)):
            got = outs[mode][acc][gi].permute(0, 3, 1, 2) - base
            err = float((got - ref).abs().max() / ref.abs().max())
            assert err < 2e-3, (gi, acc, err)
            old = outs[0][acc][gi].permute(0, 3, 1, 2) - base
            assert float((got - old).abs().max() / ref.abs().max()) < 1e-4


@pytest.mark.parametrize("shape", [(64, 256, 14, 14, 256, 1, 2), (64, 512, 7, 7, 512, 1, 2), (64, 128, 28, 28, 256, 2, 2),
                                   (64, 256, 14, 14, 512, 2, 2), (64, 64, 56, 56, 128, 2, 2), (3, 256, 14, 14, 256, 1, 2),
                                   (5, 128, 9, 11, 128, 2, 2), (2, 32, 7, 5, 128, 1, 2), (1, 512, 7, 7, 512, 1, 2),
                                   (4, 128, 28, 28, 128, 1, 2), (3, 256, 14, 14, 256, 1, 12)],
                         ids=lambda s: "x".join(map(str, s)))
def test_wgrad_ring_vs_fp32(dev, shape):
    """k_wgrad_ring (3x3 weight gradient, 128 x 288 tiles, loader waves feeding a 3-slot LDS ring,
    splits over the pixel steps sized to one workgroup per CU, slabs summed in a fixed order; one
    split writes the gradient directly) against fp32 PyTorch per view group, plain and
    accumulating, strided and ragged shapes (M not a multiple of 64) included, 2 and 12 (C5) view
    groups; and against k_conv_wgrad4 within fp32 summation-order noise."""
    import ctypes
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import conv as CV
    N, C, H, W, K, st, G = shape
    P, Q = (H + 2 - 3) // st + 1, (W + 2 - 3) // st + 1
    torch.manual_seed(N * 1000 + C + H * 10 + W + st)
    x = torch.randn(G * N, H, W, C, device=dev).bfloat16()
    dy = torch.randn(G * N, P, Q, K, device=dev).bfloat16()
    lib = L.load()
    d = CV._desc_hw(N, H, W, C, K, 3, 3, st, st, 1, 1)
    outs = {}
    try:
        for m in (0, 16):
            L.check(lib.gm_conv_set_wgrad_loop(m), "loop")
            need = lib.gm_conv2d_wgrad_grouped_scratch(ctypes.byref(d), G)
            scr = torch.empty(max(need, 16), device=dev, dtype=torch.uint8)
            res = []
            for acc in (0, 1):
                dw = torch.full((G, K, 3, 3, C), 0.5, device=dev, dtype=torch.float32)
                L.check(lib.gm_conv2d_wgrad_grouped_bf16(ctypes.byref(d), G, dy.data_ptr(), x.data_ptr(),
                                                          dw.data_ptr(), K * 9 * C, C, acc, scr.data_ptr(),
                                                          need, L.stream_of(dev)), "wgrad")
                res.append(dw)
            outs[m] = res
        torch.cuda.synchronize()
    finally:
        L.check(lib.gm_conv_set_wgrad_loop(WGRAD_LOOP_DEFAULT), "loop")
    for gi in range(G):
        xr = x[gi * N:(gi + 1) * N].float().permute(0, 3, 1, 2)
        gr = dy[gi * N:(gi + 1) * N].float().permute(0, 3, 1, 2)
        ref = torch.nn.grad.conv2d_weight(xr, (K, C, 3, 3), gr, stride=st, padding=1)
        for acc, base in ((0, 0.0), (1, 0.5)):
            got = outs[16][acc][gi].permute(0, 3, 1, 2) - base
            err = float((got - ref).abs().max() / ref.abs().max())
            assert err < 2e-3, (gi, acc, err)
            old = outs[0][acc][gi].permute(0, 3, 1, 2) - base
            assert float((got - old).abs().max() / ref.abs().max()) < 1e-4


def test_wgrad_halo64_beside_a_busy_neighbour(dev):
    """The layer-1 weight gradient repeated beside a large matmul on another stream (its
    waves share the CUs and leave their LDS contents behind): every repetition bit-identical
    and finite.  Regression: taps s = 1, 2 read halo pixels 64 / 65, which once spilled into
    the next ring slot - possibly still in flight or holding a neighbour's stale LDS data -
    and 0 x NaN turned whole gradient columns non-finite about every other repetition."""
    import ctypes
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import conv as CV
    N, H, W, C, G = 64, 56, 56, 64, 2
    torch.manual_seed(0)
    x = torch.randn(G * N, H, W, C, device=dev).bfloat16()
    dy = torch.randn(G * N, H, W, C, device=dev).bfloat16()
    lib = L.load()
    d = CV._desc_hw(N, H, W, C, C, 3, 3, 1, 1, 1, 1)
    L.check(lib.gm_conv_set_wgrad_loop(WGRAD_LOOP_DEFAULT), "loop")
    need = lib.gm_conv2d_wgrad_grouped_scratch(ctypes.byref(d), G)
    scr = torch.empty(need, device=dev, dtype=torch.uint8)
    side = torch.cuda.Stream()
    big = torch.randn(8192, 8192, device=dev)
    outs = []
    for i in range(12):
        dw = torch.empty(G, C, 3, 3, C, device=dev)
        if i:
            with torch.cuda.stream(side):
                big @ big
        L.check(lib.gm_conv2d_wgrad_grouped_bf16(ctypes.byref(d), G, dy.data_ptr(), x.data_ptr(), dw.data_ptr(),
                                                  C * 9 * C, C, 0, scr.data_ptr(), need, L.stream_of(dev)), "wgrad")
        torch.cuda.synchronize()
        outs.append(dw)
    assert torch.isfinite(outs[0]).all()
    for i, dw in enumerate(outs[1:], 1):
        assert torch.equal(dw, outs[0]), (i, int((~torch.isfinite(dw)).sum()))


@pytest.mark.parametrize("shape", [(4, 256, 14, 14, 64), (2, 64, 56, 56, 256), (3, 512, 7, 7, 2048), (1, 64, 5, 3, 128),
                                   (5, 1024, 14, 14, 256), (8, 256, 56, 56, 64, 12), (8, 64, 56, 56, 256, 12),
                                   (8, 64, 56, 56, 64, 12), (8, 2048, 7, 7, 512, 12), (8, 512, 28, 28, 128, 12)],
                         ids=lambda s: "x".join(map(str, s)))
def test_conv1x1_gemm_vs_fp32(dev, shape):
    """1x1 / s1 / p0 convolutions as plain NT GEMMs (k_gemm_ring, conv1x1.hip): forward, input
    gradient with and without the fused addend, weight gradient plain and accumulating, as
    the two-view grouped launches the trunk issues (the view groups as the GEMM batch; M not a
    multiple of the 128-row tile at 5x3 and 7x7 maps) - against fp32 PyTorch and against the
    im2col kernel (gm_conv_set_1x1_gemm(0))."""
    import ctypes
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import conv as CV
    N, C, H, W, K = shape[:5]
    G = shape[5] if len(shape) > 5 else 2  # 12: the C5 trunk's view groups
    torch.manual_seed(sum(shape))
    x = torch.randn(G * N, H, W, C, device=dev).bfloat16()
    dy = torch.randn(G * N, H, W, K, device=dev).bfloat16()
    add = torch.randn(G * N, H, W, C, device=dev).bfloat16()
    w = (torch.randn(G, K, C, device=dev) / C ** 0.5).bfloat16()  # [G][K][C] = KRSC, R = S = 1
    wt = w.transpose(1, 2).contiguous()                          # [G][C][K]
    lib = L.load()
    st = L.stream_of(dev)
    dh = CV._desc_hw(N, H, W, C, K, 1, 1, 1, 1, 0, 0)
    dd = L.ConvDesc(N, H, W, C, K, 1, 1, 1, 0)
    res = {}
    try:
        for mode in (1, 0):
            L.check(lib.gm_conv_set_1x1_gemm(mode), "1x1 gemm")
            y = torch.empty(G * N, H, W, K, device=dev, dtype=torch.bfloat16)
            L.check(lib.gm_conv2d_fwd_grouped_bf16(ctypes.byref(dh), G, x.data_ptr(), w.data_ptr(), K * C,
                                                   y.data_ptr(), 0, 0, st), "fwd")
            dx = torch.empty(G * N, H, W, C, device=dev, dtype=torch.bfloat16)
            L.check(lib.gm_conv2d_dgrad_grouped_bf16(ctypes.byref(dd), G, dy.data_ptr(), wt.data_ptr(), C * K,
                                                     dx.data_ptr(), 0, 0, 0, st), "dgrad")
            dxa = torch.empty_like(dx)
            L.check(lib.gm_conv2d_dgrad_grouped_bf16(ctypes.byref(dd), G, dy.data_ptr(), wt.data_ptr(), C * K,
                                                     dxa.data_ptr(), add.data_ptr(), 0, 0, st), "dgrad+addend")
            need = lib.gm_conv2d_wgrad_grouped_scratch(ctypes.byref(dh), G)
            scr = torch.empty(max(need, 16), device=dev, dtype=torch.uint8)
            dws = []
            for acc in (0, 1):
                dw = torch.full((G, K, C), 0.5, device=dev)
                L.check(lib.gm_conv2d_wgrad_grouped_bf16(ctypes.byref(dh), G, dy.data_ptr(), x.data_ptr(),
                                                         dw.data_ptr(), K * C, C, acc, scr.data_ptr(), need, st),
                        "wgrad")
                dws.append(dw)
            torch.cuda.synchronize()
            res[mode] = (y, dx, dxa, dws)
    finally:
        L.check(lib.gm_conv_set_1x1_gemm(2), "1x1 gemm")  # the default
    for g in range(G):
        sl = slice(g * N, (g + 1) * N)
        xf, dyf, wf = x[sl].float().reshape(-1, C), dy[sl].float().reshape(-1, K), w[g].float()
        yr, dxr, dwr = xf @ wf.t(), dyf @ wf, dyf.t() @ xf
        for mode in (1, 0):
            y, dx, dxa, dws = res[mode]
            _close(y[sl].reshape(-1, K), yr, 1e-2)
            _close(dx[sl].reshape(-1, C), dxr, 1e-2)
            _close(dxa[sl].reshape(-1, C), dxr + add[sl].float().reshape(-1, C), 1e-2)
            _close(dws[0][g], dwr, 2e-3)
            _close(dws[1][g] - 0.5, dwr, 2e-3)


@pytest.mark.parametrize("shape", [(2, 256, 56, 56, 512, 2), (3, 64, 28, 28, 128, 2), (2, 1024, 14, 14, 2048, 3),
                                   (1, 64, 15, 13, 128, 2), (2, 512, 28, 28, 1024, 12)],
                         ids=lambda s: "x".join(map(str, s)))
def test_conv1x1_s2_forward_gathers_rows(dev, shape):
    """The 1x1 / s2 downsample forward on k_gemm_ring with its A rows gathered at stride 2
    (gm_conv_set_1x1_gemm(2), the default) - plain and with the BatchNorm statistics epilogue -
    against fp32 PyTorch and the im2col kernel (mode 1); odd maps (15 x 13 -> 8 x 7)."""
    import ctypes
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import conv as CV
    N, C, H, W, K, G = shape
    P, Q = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    torch.manual_seed(sum(shape))
    x = torch.randn(G * N, H, W, C, device=dev).bfloat16()
    w = (torch.randn(G, K, C, device=dev) / C ** 0.5).bfloat16()
    lib = L.load()
    st = L.stream_of(dev)
    dh = CV._desc_hw(N, H, W, C, K, 1, 1, 2, 2, 0, 0)
    nf = lib.gm_conv2d_fwd_bn_stats_floats(ctypes.byref(dh), G)
    res = {}
    try:
        for mode in (2, 1):
            L.check(lib.gm_conv_set_1x1_gemm(mode), "1x1 gemm")
            y = torch.empty(G * N, P, Q, K, device=dev, dtype=torch.bfloat16)
            L.check(lib.gm_conv2d_fwd_grouped_bf16(ctypes.byref(dh), G, x.data_ptr(), w.data_ptr(), K * C,
                                                   y.data_ptr(), 0, 0, st), "fwd")
            ys = torch.empty_like(y)
            part = torch.zeros(max(nf, 1), device=dev)
            rows = ctypes.c_int(0)
            rc = lib.gm_conv2d_fwd_grouped_bn_stats_bf16(ctypes.byref(dh), G, x.data_ptr(), w.data_ptr(), K * C,
                                                         ys.data_ptr(), part.data_ptr(), nf, ctypes.byref(rows),
                                                         0, 0, st)
            torch.cuda.synchronize()
            res[mode] = (y, ys if rc == 0 else None, part, rows.value)
    finally:
        L.check(lib.gm_conv_set_1x1_gemm(2), "1x1 gemm")
    y2, ys2, part2, rows2 = res[2]
    assert ys2 is not None and torch.equal(ys2, y2)
    for g in range(G):
        sl = slice(g * N, (g + 1) * N)
        xs = x[sl, ::2, ::2, :].float().reshape(-1, C)
        yr = xs @ w[g].float().t()
        for mode in (2, 1):
            _close(res[mode][0][sl].reshape(-1, K), yr, 1e-2)
        # the epilogue's partial rows: per 64-channel slice, rows x [64][sum, sum of squares]
        pg = part2[g * 2 * K * (rows2 + 1):][:K * rows2 * 2].view(K // 64, rows2, 64, 2).sum(1).reshape(K, 2)
        yv = y2[sl].float().reshape(-1, K)
        _close(pg[:, 0], yv.sum(0), 1e-4)
        _close(pg[:, 1], (yv * yv).sum(0), 1e-4)


@pytest.mark.parametrize("shape", [(2, 256, 56, 56, 512, 2), (3, 64, 28, 28, 128, 2), (1, 64, 15, 13, 128, 2),
                                   (2, 512, 28, 28, 1024, 12)],
                         ids=lambda s: "x".join(map(str, s)))
def test_conv1x1_s2_input_gradient_scatters_rows(dev, shape):
    """The 1x1 / s2 downsample's input gradient on k_gemm_ring: dy rows read densely, output rows
    scattered to the even pixels, the odd ones zero / the join addend (plain, masked, in place) -
    against fp32 PyTorch and the im2col kernel (mode 1); the odd pixels exactly zero / the addend."""
    import ctypes
    from greedy_multimodal_learning_amd import _lib as L
    N, C, H, W, K, G = shape
    P, Q = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    torch.manual_seed(sum(shape) + 1)
    dy = torch.randn(G * N, P, Q, K, device=dev).bfloat16()
    w = (torch.randn(G, K, C, device=dev) / K ** 0.5).bfloat16()
    wt = w.transpose(1, 2).contiguous()  # [G][C][K]
    add = torch.randn(G * N, H, W, C, device=dev).bfloat16()
    mask = torch.randint(0, 256, (add.numel() // 8,), device=dev, dtype=torch.uint8)
    lib = L.load()
    st = L.stream_of(dev)
    dd = L.ConvDesc(N, H, W, C, K, 1, 1, 2, 0)
    res = {}
    try:
        for mode in (2, 1):
            L.check(lib.gm_conv_set_1x1_gemm(mode), "1x1 gemm")
            dx = torch.full((G * N, H, W, C), 7.0, device=dev, dtype=torch.bfloat16)
            L.check(lib.gm_conv2d_dgrad_grouped_bf16(ctypes.byref(dd), G, dy.data_ptr(), wt.data_ptr(), C * K,
                                                     dx.data_ptr(), 0, 0, 0, st), "dgrad")
            dxa = add.clone()  # in place
            L.check(lib.gm_conv2d_dgrad_grouped_bf16(ctypes.byref(dd), G, dy.data_ptr(), wt.data_ptr(), C * K,
                                                     dxa.data_ptr(), dxa.data_ptr(), 0, 0, st), "dgrad in place")
            dxm = torch.empty_like(dx)
            L.check(lib.gm_conv2d_dgrad_grouped_masked_bf16(ctypes.byref(dd), G, dy.data_ptr(), wt.data_ptr(),
                                                            C * K, dxm.data_ptr(), add.data_ptr(), mask.data_ptr(),
                                                            0, 0, st), "dgrad masked")
            torch.cuda.synchronize()
            res[mode] = (dx, dxa, dxm)
    finally:
        L.check(lib.gm_conv_set_1x1_gemm(2), "1x1 gemm")
    bits = ((mask.to(torch.int32)[:, None] >> torch.arange(8, device=dev)) & 1).reshape(add.shape).bool()
    madd = torch.where(bits, add, torch.zeros((), dtype=add.dtype, device=dev))
    for i in range(3):  # (the im2col kernel may split K: another fp32 order)
        _close(res[2][i], res[1][i], 8e-3)
    for g in range(G):
        sl = slice(g * N, (g + 1) * N)
        ref = torch.zeros(N, H, W, C, device=dev)
        ref[:, ::2, ::2, :] = (dy[sl].float().reshape(-1, K) @ w[g].float()).reshape(N, P, Q, C)
        _close(res[2][0][sl], ref, 1e-2)
        _close(res[2][1][sl], ref + add[sl].float(), 1e-2)
        _close(res[2][2][sl], ref + madd[sl].float(), 1e-2)
        odd = torch.ones(H, W, dtype=torch.bool, device=dev)
        odd[::2, ::2] = False
        assert torch.equal(res[2][0][sl][:, odd], torch.zeros_like(res[2][0][sl][:, odd]))
        assert torch.equal(res[2][2][sl][:, odd], madd[sl][:, odd])


@pytest.mark.parametrize("case", [("bf16_cl", 2, 4, 224, 224), ("bf16_cl", 3, 2, 37, 30), ("f32_nchw", 2, 3, 64, 64),
                                  ("bf16_nchw", 2, 2, 31, 40), ("f32_cl", 4, 1, 19, 22)],
                         ids=lambda c: "x".join(map(str, c)))
def test_stem_pack_grouped_matches_per_view(dev, case):
    """gm_stem_pack_grouped_bf16 (every view in one launch: whole-vector row loads for channels-
    last bf16 views, element loads otherwise) == one gm_stem_pack_bf16 per view, bit for bit,
    for the bench's view-major channels-last batch and NCHW / fp32 inputs, ragged sizes."""
    from greedy_multimodal_learning_amd.conv import _stem_geom, stem_pack, stem_pack_grouped
    kind, G, N, H, W = case
    g = torch.Generator().manual_seed(G * 100 + H)
    dt = torch.bfloat16 if kind.startswith("bf16") else torch.float32
    if kind.endswith("_cl"):  # view-major, channels-last storage seen as [N, G, 3, H, W]
        x = torch.randn(G, N, H, W, 3, generator=g).to(dt).to(dev).permute(1, 0, 4, 2, 3)
    else:
        x = torch.randn(N, G, 3, H, W, generator=g).to(dt).to(dev)
    ws = [torch.randn(64, 3, 7, 7, generator=g).to(dev) for _ in range(G)]
    ws[0] = ws[0].contiguous(memory_format=torch.channels_last)  # strided weight (the model's layout)
    P, Q, Sp, Hp, Wp = _stem_geom(H, W, 7, 7, 3)
    xp = torch.full((G * N, Hp, Wp // 2, 8), 7.0, device=dev, dtype=torch.bfloat16)
    wp = torch.full((G, 64, 7, Sp, 8), 7.0, device=dev, dtype=torch.bfloat16)
    stem_pack_grouped([x[:, i] for i in range(G)], ws, 3, xp, wp)
    for i in range(G):
        rx = torch.empty(N, Hp, Wp // 2, 8, device=dev, dtype=torch.bfloat16)
        rw = torch.empty(64, 7, Sp, 8, device=dev, dtype=torch.bfloat16)
        stem_pack(x[:, i], ws[i], 3, xp=rx, wp=rw)
        assert torch.equal(xp[i * N:(i + 1) * N].view(torch.int16), rx.view(torch.int16)), f"view {i} input"
        assert torch.equal(wp[i].view(torch.int16), rw.view(torch.int16)), f"view {i} weight"
