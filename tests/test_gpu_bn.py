"""HIP BatchNorm(+residual+ReLU) kernels vs a plain PyTorch fp32 reference of the
same op (F.batch_norm on the bf16-rounded input), forward, backward, running
statistics, eval mode, in-place gradient delivery and determinism."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last
SHAPES = [(4, 64, 16, 16), (2, 128, 7, 7), (3, 8, 5, 5), (64, 512, 7, 7), (8, 256, 14, 14), (2, 2048, 4, 4),
          (16, 64, 56, 56)]


def _ref(x, w, b, rm, rv, res, relu, momentum=0.1, eps=1e-5):
    """fp32 autograd reference; returns y, running stats after the update."""
    rm, rv = rm.clone(), rv.clone()
    y = F.batch_norm(x, rm, rv, w, b, training=True, momentum=momentum, eps=eps)
    if res is not None:
        y = y + res
    if relu:
        y = F.relu(y)
    return y, rm, rv


def _inputs(shape, seed, res):
    g = torch.Generator(device="cuda").manual_seed(seed)
    N, C, H, W = shape
    x = (torch.randn(shape, device="cuda", generator=g) * 1.7 + 0.3).bfloat16().contiguous(memory_format=CL)
    r = torch.randn(shape, device="cuda", generator=g).bfloat16().contiguous(memory_format=CL) if res else None
    w = torch.rand(C, device="cuda", generator=g) + 0.5
    b = torch.randn(C, device="cuda", generator=g) * 0.1
    rm = torch.randn(C, device="cuda", generator=g) * 0.1
    rv = torch.rand(C, device="cuda", generator=g) + 0.5
    dy = torch.randn(shape, device="cuda", generator=g).bfloat16().contiguous(memory_format=CL)
    return x, r, w, b, rm, rv, dy


@pytest.fixture
def fused_mode():
    """Switch the single-launch BatchNorm mode (gm_bn_set_fused_mode); restores 2."""
    from greedy_multimodal_learning_amd import _lib as L
    yield lambda m: L.check(L.load().gm_bn_set_fused_mode(int(m)), "gm_bn_set_fused_mode")
    L.load().gm_bn_set_fused_mode(2)


def _rel(a, b):
    return (a.float() - b.float()).abs().max().item() / max(b.float().abs().max().item(), 1e-6)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("res,relu", [(False, False), (False, True), (True, True)])
def test_bn_train_fwd_bwd(shape, res, relu):
    from greedy_multimodal_learning_amd.bn import GMBatchNorm2d
    x, r, w, b, rm, rv, dy = _inputs(shape, 7 + shape[1], res)
    C = shape[1]
    m = GMBatchNorm2d(C).cuda().to(memory_format=CL)
    with torch.no_grad():
        m.weight.copy_(w)
        m.bias.copy_(b)
        m.running_mean.copy_(rm)
        m.running_var.copy_(rv)
    xg = x.clone().requires_grad_(True)
    rg = r.clone().requires_grad_(True) if res else None
    y = m(xg, residual=rg, relu=relu)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=CL)
    y.backward(dy)

    xr = x.float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    rr = r.float().requires_grad_(True) if res else None
    yr, rm_r, rv_r = _ref(xr, wr, br, rm, rv, rr, relu)
    yr.backward(dy.float())

    assert _rel(y, yr) < 1e-2
    assert torch.allclose(m.running_mean, rm_r, rtol=1e-4, atol=1e-5)
    assert torch.allclose(m.running_var, rv_r, rtol=1e-4, atol=1e-5)
    assert int(m.num_batches_tracked) == 1
    assert _rel(xg.grad, xr.grad) < 1.5e-2
    assert _rel(m.weight.grad, wr.grad) < 2e-3
    assert _rel(m.bias.grad, br.grad) < 2e-3
    if res:
        assert _rel(rg.grad, rr.grad) < 1e-2


def test_bn_deterministic_and_eval():
    from greedy_multimodal_learning_amd.bn import GMBatchNorm2d
    shape = (32, 64, 28, 28)
    x, r, w, b, rm, rv, dy = _inputs(shape, 3, True)
    outs = []
    for _ in range(2):
        m = GMBatchNorm2d(64).cuda()
        xg = x.clone().requires_grad_(True)
        y = m(xg, residual=r, relu=True)
        y.backward(dy)
        outs.append((y, xg.grad, m.weight.grad.clone(), m.running_var.clone()))
    for a, b2 in zip(*outs):
        assert torch.equal(a, b2)
    # eval: running statistics
    m.eval()
    with torch.no_grad():
        ye = m(x, residual=r, relu=True)
        yr = F.relu(F.batch_norm(x.float(), m.running_mean, m.running_var, m.weight, m.bias, False) + r.float())
    assert _rel(ye, yr) < 1e-2


def test_bn_grad_sink_in_place():
    """Engine mode: weight/bias gradients land in .grad in place (overwrite, then
    accumulate on a second use within the step) and the hook fires."""
    from greedy_multimodal_learning_amd.bn import GMBatchNorm2d
    from greedy_multimodal_learning_amd.gradsink import GradSink
    shape = (8, 128, 14, 14)
    x, _, w, b, rm, rv, dy = _inputs(shape, 5, False)
    m = GMBatchNorm2d(128).cuda()
    fired = []
    m.weight.grad = torch.full_like(m.weight, 7.0)  # stale content must be overwritten
    m.bias.grad = torch.full_like(m.bias, 7.0)
    sink = GradSink(m.parameters(), on_ready=fired.append)
    sink.begin_step()
    y = m(x.clone().requires_grad_(True), relu=True)
    y.backward(dy)
    g1 = m.weight.grad.clone()
    y2 = m(x.clone().requires_grad_(True), relu=True)
    y2.backward(dy)
    sink.end_step()
    assert len(fired) == 4
    sink.detach()
    m2 = GMBatchNorm2d(128).cuda()
    y3 = m2(x.clone().requires_grad_(True), relu=True)
    y3.backward(dy)
    assert torch.allclose(g1, m2.weight.grad, rtol=0, atol=0)
    assert torch.allclose(m.weight.grad, 2 * m2.weight.grad, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("shape", SHAPES)
def test_bn_relu_mask_from_x_equals_y_mask(shape, monkeypatch):
    """ReLU BN without a residual: the backward's mask recomputed from x and the
    forward's coefficients (x*sc + sh > 0) == the mask read from y, bit for bit."""
    from greedy_multimodal_learning_amd import bn as B
    x, _, w, b, rm, rv, dy = _inputs(shape, 11 + shape[0], False)
    C = shape[1]
    outs = []
    for maskx in (False, True):
        monkeypatch.setattr(B, "MASK_FROM_X", maskx)
        m = B.GMBatchNorm2d(C).cuda().to(memory_format=CL)
        with torch.no_grad():
            m.weight.copy_(w)
            m.bias.copy_(b)
        xg = x.clone().requires_grad_(True)
        y = m(xg, relu=True)
        y.backward(dy)
        outs.append((y, xg.grad, m.weight.grad, m.bias.grad))
    for a, b2 in zip(*outs):
        assert torch.equal(a, b2)


@pytest.mark.parametrize("mode", ["1", "2"])  # register-held strips only / + the streaming variant
@pytest.mark.parametrize("shape", [(64, 64, 112, 112), (64, 64, 56, 56), (64, 128, 28, 28), (64, 256, 14, 14),
                                   (64, 512, 7, 7), (3, 8, 5, 5), (7, 64, 9, 11)])
@pytest.mark.parametrize("res,relu", [(False, False), (False, True), (True, True)])
def test_bn_fused_forward_equals_two_kernel_forward(shape, res, relu, mode, fused_mode):
    """The single-launch forward (co-resident blocks, in-launch coefficient hand-off)
    == the reduce + apply pair (its own row partition: fp32 partial sums in another
    grouping, so y within one bf16 ulp, running stats to 1e-5), and bit-identical
    to itself across launches."""
    from greedy_multimodal_learning_amd.bn import GMBatchNorm2d
    x, r, w, b, rm, rv, dy = _inputs(shape, 13 + shape[2], res)
    outs = []
    for fused in ("0", mode, mode):  # the fused path twice: its generation words advance
        fused_mode(fused)
        m = GMBatchNorm2d(shape[1]).cuda().to(memory_format=CL)
        with torch.no_grad():
            m.weight.copy_(w)
            m.bias.copy_(b)
        y = m(x.clone().requires_grad_(True), residual=r, relu=relu)
        outs.append((y, m.running_mean.clone(), m.running_var.clone()))
    for a, b2 in zip(outs[1], outs[2]):
        assert torch.equal(a, b2)
    y0, y1 = outs[0][0].float(), outs[1][0].float()
    assert ((y0 - y1).abs() <= 2 ** -7 * y0.abs().clamp_min(1e-3)).all()
    for a, b2 in zip(outs[0][1:], outs[1][1:]):
        torch.testing.assert_close(b2, a, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("mode", ["1", "2"])
@pytest.mark.parametrize("shape", [(64, 64, 112, 112), (64, 64, 56, 56), (64, 128, 28, 28), (64, 256, 14, 14),
                                   (64, 512, 7, 7), (3, 8, 5, 5), (7, 64, 9, 11)])
@pytest.mark.parametrize("res,relu,maskx", [(False, False, True), (False, True, True), (False, True, False),
                                            (True, True, True)])
def test_bn_fused_backward_equals_two_kernel_backward(shape, res, relu, maskx, mode, monkeypatch, fused_mode):
    """The single-launch backward == the reduce + apply_bwd pair (own row partition:
    dgamma/dbeta to 1e-5, dx/dres within one bf16 ulp of the larger magnitude) and
    bit-identical to itself across launches."""
    from greedy_multimodal_learning_amd import bn as B
    monkeypatch.setattr(B, "MASK_FROM_X", maskx)
    x, r, w, b, rm, rv, dy = _inputs(shape, 17 + shape[3], res)
    outs = []
    for fused in ("0", mode, mode):
        fused_mode(0)  # same forward for all three
        m = B.GMBatchNorm2d(shape[1]).cuda().to(memory_format=CL)
        with torch.no_grad():
            m.weight.copy_(w)
            m.bias.copy_(b)
        xg = x.clone().requires_grad_(True)
        rg = r.clone().requires_grad_(True) if res else None
        y = m(xg, residual=rg, relu=relu)
        fused_mode(fused)
        y.backward(dy)
        outs.append((xg.grad, rg.grad if res else None, m.weight.grad, m.bias.grad))
    for a, b2 in zip(outs[1], outs[2]):
        assert (a is None and b2 is None) or torch.equal(a, b2)
    for k in (0, 1):
        if outs[0][k] is None:
            continue
        a, b2 = outs[0][k].float(), outs[1][k].float()
        tol = 2 ** -7 * torch.maximum(a.abs(), b2.abs()) + 1e-3 * a.abs().max()
        assert ((a - b2).abs() <= tol).all()
    for k in (2, 3):
        torch.testing.assert_close(outs[1][k], outs[0][k], rtol=1e-4, atol=1e-4 * outs[0][k].abs().max().item())


def test_bn_fused_spin_timeout_faults_loudly(fused_mode):
    """A coefficient hand-off that runs out of its poll budget (forced: budget 1 poll)
    must never apply stale coefficients: the fault word is raised and the affected
    outputs are NaN; the engine's sync point raises GreedyMMLError."""
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd.bn import GMBatchNorm2d
    lib = L.load()
    L.device_faults(clear=True)
    shape = (64, 64, 56, 56)  # hundreds of blocks: early arrivals poll before the last ticket
    x, r, w, b, rm, rv, dy = _inputs(shape, 21, False)
    fused_mode(2)
    m = GMBatchNorm2d(64).cuda()
    ref = m(x.clone(), relu=True).float()
    m = GMBatchNorm2d(64).cuda()
    try:
        L.check(lib.gm_set_spin_limit(1), "gm_set_spin_limit")
        y = m(x.clone(), relu=True).float()
        torch.cuda.synchronize()
    finally:
        lib.gm_set_spin_limit(0)
    faults = L.device_faults()
    if faults & L.GM_FAULT_BN_SPIN:
        assert torch.isnan(y).any()  # poisoned, never silently stale
        with pytest.raises(L.GreedyMMLError, match="BatchNorm"):
            L.check_device_faults()
    else:  # every block happened to see the coefficients at its first poll: exact result
        assert torch.equal(y, ref)
    assert L.device_faults() == 0  # cleared by check_device_faults
    assert torch.equal(m(x.clone(), relu=True).float(), ref)  # default budget: healthy again


def test_bn_fused_concurrent_streams_match_serial(fused_mode):
    """More concurrent single-launch BatchNorms than the default reservation (6 streams
    x forward + backward, view trunks of a 6-view model) == the same launches one after
    another, with no fault: the planner's co-residency cap holds (gm_bn_set_concurrency
    raised by the N-view streams)."""
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd.bn import GMBatchNorm2d
    from greedy_multimodal_learning_amd.streams import reserve_concurrency
    L.device_faults(clear=True)
    fused_mode(2)
    n = 6
    reserve_concurrency(n + 2)
    shapes = [(64, 64, 56, 56), (64, 128, 28, 28), (64, 256, 14, 14)]
    ins = [_inputs(shapes[i % 3], 40 + i, i % 2 == 0) for i in range(n)]

    def run(i):
        x, r, w, b, rm, rv, dy = ins[i]
        m = GMBatchNorm2d(x.shape[1]).cuda()
        xg = x.clone().requires_grad_(True)
        y = m(xg, residual=r, relu=True)
        y.backward(dy)
        return y, xg.grad, m.weight.grad

    serial = [run(i) for i in range(n)]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(n)]
    outs = [None] * n
    for i, s in enumerate(streams):
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            outs[i] = run(i)
    torch.cuda.synchronize()
    assert L.device_faults() == 0
    for a, b2 in zip(serial, outs):
        for u, v in zip(a, b2):
            assert torch.equal(u, v)


@pytest.mark.parametrize("shape", [(4, 64, 16, 16), (2, 64, 112, 112), (3, 8, 9, 7), (2, 128, 15, 14)])
def test_bn_relu_maxpool_fused_stem(shape, fused_mode):
    """The stem's relu(bn1(x)) -> MaxPool2d(3, 2, 1) on the fused path (statistics launch
    + pool applying the affine + ReLU on the fly): bit-identical forward and pool
    indices to bn(x, relu=True) on the two-kernel BN path followed by the plain pool
    (same statistics partition), running statistics and num_batches_tracked updated,
    gradients equal to the composed modules and within bf16 tolerance of fp32."""
    from greedy_multimodal_learning_amd import bn as B
    from greedy_multimodal_learning_amd.pool import GMMaxPool2d
    x, _, w, b, rm, rv, _ = _inputs(shape, 11 + shape[2], False)
    N, C, H, W = shape
    pool = GMMaxPool2d(kernel_size=3, stride=2, padding=1)
    P, Q = (H + 2 - 3) // 2 + 1, (W + 2 - 3) // 2 + 1
    g = torch.Generator(device="cuda").manual_seed(5)
    dy = torch.randn(N, C, P, Q, device="cuda", generator=g).bfloat16().contiguous(memory_format=CL)
    outs = []
    for fuse in (True, False):
        m = B.GMBatchNorm2d(C).cuda().to(memory_format=CL)
        with torch.no_grad():
            m.weight.copy_(w)
            m.bias.copy_(b)
            m.running_mean.copy_(rm)
            m.running_var.copy_(rv)
        xg = x.clone().requires_grad_(True)
        old = B.FUSE_POOL
        B.FUSE_POOL = fuse
        try:
            fused_mode(0)  # the composed path's BN on the two-kernel partition (the fused stem's)
            y = m.relu_maxpool(xg, pool)
            y.backward(dy)
        finally:
            B.FUSE_POOL = old
        outs.append((y, xg.grad, m.weight.grad, m.bias.grad, m.running_mean.clone(), m.running_var.clone(),
                     int(m.num_batches_tracked), type(y.grad_fn).__name__))
    (yf, dxf, dwf, dbf, rmf, rvf, nbf, fnf), (yc, dxc, dwc, dbc, rmc, rvc, nbc, _) = outs
    assert "BNReluPool" in fnf
    assert torch.equal(yf, yc)
    assert torch.equal(rmf, rmc) and torch.equal(rvf, rvc) and nbf == nbc == 1
    assert torch.equal(dxf, dxc) and torch.equal(dwf, dwc) and torch.equal(dbf, dbc)
    xr = x.float().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    # the pooled values are bf16 in both paths: pool the bf16-rounded activation so that
    # window ties (and so the argmax the gradient follows) match
    zr = F.relu(F.batch_norm(xr, rm.clone(), rv.clone(), wr, br, training=True))
    yr = F.max_pool2d(zr.bfloat16().float(), 3, 2, 1)
    yr.backward(dy.float())
    assert _rel(yf, yr) < 1e-2
    assert _rel(dxf, xr.grad) < 2e-2
    assert _rel(dwf, wr.grad) < 5e-3 and _rel(dbf, br.grad) < 5e-3
