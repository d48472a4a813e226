"""Kernel-level parity through the C ABI: GEMM, spatial reduce, channel scale,
running average and the group-norm (+SGD) pass against fp32/fp64 references."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (3, 5, 7), (64, 512, 1024), (64, 128, 256),
                                   (256, 512, 64), (17, 33, 129), (1, 300, 64), (512, 1024, 64)])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_gemm_f32(dev, M, N, K, act):
    from greedy_multimodal_learning_amd import ops
    g = torch.Generator().manual_seed(M * 1000 + N + K)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    y = ops.linear(x.to(dev), w.to(dev), b.to(dev), act=act).cpu()
    ref = (x.double() @ w.double().T + b.double())
    if act == 1:
        ref = ref.clamp_min(0)
    elif act == 2:
        ref = torch.sigmoid(ref)
    np.testing.assert_allclose(y.numpy(), ref.numpy(), rtol=1e-4, atol=1e-5 * K ** 0.5)


def test_gemm_segments_strides_ones_mask_accumulate(dev):
    from greedy_multimodal_learning_amd import ops
    from greedy_multimodal_learning_amd.ops import ONES, Op
    g = torch.Generator().manual_seed(3)
    B, C1, C2, N = 5, 24, 40, 36
    a1, a2 = torch.randn(B, C1, generator=g), torch.randn(C2, generator=g)
    w = torch.randn(N, C1 + C2, generator=g)
    mask = (torch.randn(B, N, generator=g) > 0).float()
    c0 = torch.randn(B, N, generator=g)
    A1, A2, W, MK, Cd = (t.to(dev).contiguous() for t in (a1, a2, w, mask, c0))
    # C += relu-masked( a1 @ W[:, :C1]^T + broadcast(a2) @ W[:, C1:]^T )
    ops.gemm([dict(M=B, N=N, segs=[(C1, Op(A1, C1, 1), Op(W, 1, C1 + C2)),
                                   (C2, Op(A2, 0, 1), Op(W, 1, C1 + C2, off=C1))],
                   C=Cd, ld_c=N, mask=MK, ld_mask=N, accumulate=1)], dev)
    ref = c0 + (a1 @ w[:, :C1].T + a2[None] @ w[:, C1:].T) * (mask > 0)
    np.testing.assert_allclose(Cd.cpu().numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)
    # column sums via the ones operand
    out = torch.empty(1, N, device=dev)
    ops.gemm([dict(M=1, N=N, segs=[(B, ONES, Op(MK, N, 1))], C=out, ld_c=N)], dev)
    np.testing.assert_allclose(out.cpu().numpy()[0], mask.sum(0).numpy(), rtol=1e-6)


@pytest.mark.parametrize("M,N,K,acc", [(2048, 24576, 32, 1), (300, 5000, 32, 0), (1004, 1028, 100, 1),
                                       (64, 16384, 7, 0), (1000, 1027, 100, 1)])
def test_gemm_outer_product_shapes(dev, M, N, K, acc):
    """The outer-product kernel (k_gemm_outer: K <= 128, M x N >= 2^20 - the C5 MMTM weight
    gradients, fc_squeeze's dW[2048][24576] = dz^T . sq at K = B = 32) against fp64, with the
    strided A^T operand the MMTM backward passes (Op(dz, 1, M)), accumulating into C, ragged
    edges (a partial row group, a partial column chunk), a K tail, and a shape whose unaligned
    rows fall back to k_gemm_f32; equal within fp32 summation order to k_gemm_f32 (form bit 9)."""
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import ops
    from greedy_multimodal_learning_amd.ops import Op
    g = torch.Generator().manual_seed(M + N + K)
    dz = torch.randn(K, M, generator=g)        # the GEMM's A = dz^T (A[m, k] = dz[k, m])
    sq = torch.randn(K, N, generator=g)
    c0 = torch.randn(M, N, generator=g) if acc else torch.zeros(M, N)
    ref = c0.double() + dz.double().T @ sq.double()
    outs = []
    try:
        for form in (1, 1 | 512):
            L.check(L.load().gm_gemm_set_form(form), "gemm form")
            C = c0.to(dev).contiguous()
            ops.gemm([dict(M=M, N=N, segs=[(K, Op(dz.to(dev), 1, M), Op(sq.to(dev), N, 1))], C=C, ld_c=N,
                           accumulate=acc)], dev)
            outs.append(C.cpu())
    finally:
        L.check(L.load().gm_gemm_set_form(1), "gemm form")
    scale = float(ref.abs().max())
    for o in outs:
        assert float((o.double() - ref).abs().max()) <= 1e-5 * scale
    assert float((outs[0] - outs[1]).abs().max()) <= 1e-5 * scale


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("layout", ["nchw", "nhwc"])
@pytest.mark.parametrize("B,C,H,W", [(2, 128, 28, 28), (3, 256, 14, 14), (64, 512, 7, 7),
                                     (1, 8, 1, 1), (5, 64, 3, 5), (7, 128, 1, 3),
                                     (3, 2048, 7, 7), (2, 4096, 2, 3)])  # ResNet-50 widths: several channel slabs
def test_spatial_reduce_and_scale(dev, dtype, layout, B, C, H, W):
    from greedy_multimodal_learning_amd import ops, _lib as L
    g = torch.Generator().manual_seed(B * C + H)
    x = torch.randn(B, C, H, W, generator=g).to(dtype)
    dy = torch.randn(B, C, H, W, generator=g).to(dtype)
    e = torch.rand(B, C, generator=g)
    fmt = torch.channels_last if layout == "nhwc" else torch.contiguous_format
    X, DY = x.to(dev).contiguous(memory_format=fmt), dy.to(dev).contiguous(memory_format=fmt)
    lay = ops.act_layout(X)
    dt = ops._DT[dtype]
    HW = H * W
    out = torch.empty(B, 2 * C, device=dev)
    E = e.to(dev)
    ops.spatial_reduce([dict(x=X, C=C, HW=HW, out=out, ld_out=2 * C, scale=1.0 / HW),
                        dict(x=X, dy=DY, C=C, HW=HW, out=out, out_off=C, ld_out=2 * C, e=E, ld_e=C)][:1],
                       B, dt, lay, dev)
    ops.spatial_reduce([dict(x=X, dy=DY, C=C, HW=HW, out=out, out_off=C, ld_out=2 * C, e=E, ld_e=C)],
                       B, dt, lay, dev)
    xf, df = x.double(), dy.double()
    ref_sq = xf.mean((2, 3))
    ref_da = (xf * df).sum((2, 3)) * e.double() * (1 - e.double())
    o = out.cpu().double()
    np.testing.assert_allclose(o[:, :C].numpy(), ref_sq.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(o[:, C:].numpy(), ref_da.numpy(), rtol=1e-4, atol=1e-4)
    # scale (fwd) and apply (bwd)
    s = torch.rand(B, C, generator=g)
    a = torch.randn(B, C, generator=g)
    Y, DX = torch.empty_like(X), torch.empty_like(X)
    S, A = s.to(dev), a.to(dev)
    ops.channel_scale([dict(x=X, y=Y, C=C, HW=HW, s=S, ld_s=C)], B, dt, lay, dev)
    ops.channel_scale([dict(x=DY, y=DX, C=C, HW=HW, s=S, ld_s=C, a=A, ld_a=C, alpha=1.0 / HW)],
                      B, dt, lay, dev)
    ref_y = (xf * s.double()[:, :, None, None]).to(dtype).double()
    ref_dx = (df * s.double()[:, :, None, None] + a.double()[:, :, None, None] / HW).to(dtype).double()
    tol = 1e-6 if dtype == torch.float32 else 8e-3
    np.testing.assert_allclose(Y.cpu().double().numpy(), ref_y.numpy(), rtol=tol, atol=tol)
    np.testing.assert_allclose(DX.cpu().double().numpy(), ref_dx.numpy(), rtol=tol, atol=tol)
    # broadcast row (curation): ld_s = 0
    ops.channel_scale([dict(x=X, y=Y, C=C, HW=HW, s=S, ld_s=0)], B, dt, lay, dev)
    ref_b = (xf * s.double()[0][None, :, None, None]).to(dtype).double()
    np.testing.assert_allclose(Y.cpu().double().numpy(), ref_b.numpy(), rtol=tol, atol=tol)


def test_running_avg(dev):
    from greedy_multimodal_learning_amd import ops
    e = torch.rand(6, 40)
    rv, rs = torch.rand(40), torch.rand(40)
    nv, ns = ops.running_avg(e.to(dev), rv.to(dev), rs.to(dev), 7)
    m = e.mean(0)
    np.testing.assert_allclose(nv.cpu().numpy(), ((m + rv * 7) / 8).numpy(), rtol=1e-6)
    np.testing.assert_allclose(ns.cpu().numpy(), ((m + rs * 7) / 8).numpy(), rtol=1e-6)


@pytest.mark.parametrize("lr", [0.0, 0.1])
def test_group_sumsq_and_fused_sgd(dev, lr):
    from greedy_multimodal_learning_amd.callbacks import GroupNorms
    g = torch.Generator().manual_seed(1)
    shapes = {"net_view_0.a": (3, 5), "net_view_0.b": (40000,), "net_view_1.c": (7,),
              "net_view_1.d": (100, 333), "mmtm2.fc_squeeze.weight": (16, 32),
              "mmtm2.fc_visual.bias": (16,), "mmtm3.fc_skeleton.weight": (64, 65),
              "net_view_1.e": (1,)}
    params = []
    for n, s in shapes.items():
        p = torch.nn.Parameter(torch.randn(*s, generator=g).to(dev))
        p.grad = torch.randn(*s, generator=g).to(dev)
        params.append((n, p))
    before = {n: (p.detach().double().cpu(), p.grad.double().cpu()) for n, p in params}
    gn = GroupNorms(params, ["net_view_0", "net_view_1"], ["visual", "skeleton"])
    out = gn.sums(grad_scale=0.5, lr=lr).cpu().numpy()
    ref = np.zeros(8)
    for n, (w, gr) in before.items():
        gr = gr * 0.5
        groups = []
        if "mmtm" in n:
            groups = [2] if "visual" in n else [3] if "skeleton" in n else [2, 3]
        else:
            groups = [0] if "net_view_0" in n else [1]
        for k in groups:
            ref[2 * k] += float((w ** 2).sum())
            ref[2 * k + 1] += float((gr ** 2).sum())
    np.testing.assert_allclose(out, ref, rtol=1e-6)
    for n, p in params:
        w, gr = before[n]
        np.testing.assert_allclose(p.detach().cpu().double().numpy(), (w - lr * 0.5 * gr).numpy(),
                                   rtol=1e-6, atol=1e-7)


def test_group_sumsq_twelve_branches(dev):
    """The C5 gate: 12 branches x (main, bypass) = 24 groups (the 32-group kernel)."""
    from greedy_multimodal_learning_amd.callbacks import GroupNorms, group_masks
    g = torch.Generator().manual_seed(3)
    V = 12
    bn = [f"net_view_{i}" for i in range(V)]
    mn = [f"fc_excite.{i}." for i in range(V)]
    params = []
    for i in range(V):
        for n, s in ((f"net_view_{i}.conv.weight", (64, 3, 3, 3)), (f"net_view_{i}.bn.bias", (64,))):
            params.append((n, torch.nn.Parameter(torch.randn(*s, generator=g).to(dev))))
        params.append((f"mmtm4.fc_excite.{i}.weight", torch.nn.Parameter(torch.randn(32, 16, generator=g).to(dev))))
    params.append(("mmtm4.fc_squeeze.weight", torch.nn.Parameter(torch.randn(16, 384, generator=g).to(dev))))
    for _, p in params:
        p.grad = torch.randn(p.shape, generator=g).to(dev)
    gn = GroupNorms(params, bn, mn)
    out = gn.sums().cpu().numpy()
    masks = group_masks([n for n, _ in params], bn, mn)
    ref = np.zeros(4 * V)
    for (n, p), m in zip(params, masks):
        for k in range(2 * V):
            if (m >> k) & 1:
                ref[2 * k] += float((p.detach().double() ** 2).sum())
                ref[2 * k + 1] += float((p.grad.double() ** 2).sum())
    assert masks[0] == 1 and masks[3 * 10] == 1 << 10  # net_view_10 is not net_view_1
    np.testing.assert_allclose(out, ref, rtol=1e-6)


@pytest.mark.parametrize("V", [12, 2])
def test_group_sumsq_long_chunks(dev, V):
    """Totals above 16384 x 4096 elements take longer chunks (fewer finalize rows); the
    many-group form (V=12) flushes per mask run.  Odd tensor sizes exercise the scalar
    heads/tails at every chunk boundary; reference = fp64 sums on the device."""
    from greedy_multimodal_learning_amd.callbacks import GroupNorms, group_masks
    g = torch.Generator(device=dev).manual_seed(5)
    bn = [f"net_view_{i}" for i in range(V)]
    mn = [f"fc_excite.{i}." for i in range(V)]
    per = 72_000_000 // V
    params = []
    for i in range(V):
        for n, s in ((f"net_view_{i}.conv.weight", (per - 1001,)), (f"net_view_{i}.bn.bias", (1001,)),
                     (f"net_view_{i}.bn.weight", (3,))):
            params.append((n, torch.nn.Parameter(torch.randn(*s, generator=g, device=dev))))
        params.append((f"mmtm4.fc_excite.{i}.weight", torch.nn.Parameter(torch.randn(333, 17, generator=g, device=dev))))
    params.append(("mmtm4.fc_squeeze.weight", torch.nn.Parameter(torch.randn(1000, 77, generator=g, device=dev))))
    for _, p in params:
        p.grad = torch.randn(p.shape, generator=g, device=dev)
    masks = group_masks([n for n, _ in params], bn, mn)
    ref = torch.zeros(4 * V, dtype=torch.float64, device=dev)
    for (n, p), m in zip(params, masks):
        sw = (p.detach().double() ** 2).sum()
        sg = ((p.grad.double() * 0.5) ** 2).sum()
        for k in range(2 * V):
            if (m >> k) & 1:
                ref[2 * k] += sw
                ref[2 * k + 1] += sg
    want = [(p.detach() - 0.01 * 0.5 * p.grad).clone() for _, p in params]
    gn = GroupNorms(params, bn, mn)
    out = gn.sums(grad_scale=0.5, lr=0.01)
    np.testing.assert_allclose(out.cpu().numpy(), ref.cpu().numpy(), rtol=1e-6)
    for (_, p), w in zip(params, want):
        torch.testing.assert_close(p.detach(), w, rtol=1e-6, atol=1e-7)

