"""Per-shape launch table of the bf16 ResNet-18 trunk at the step's batch, as the step
launches it: the two views' trunks batched into grouped launches (vtrunk.py; --groups 1
for one view alone): every convolution pass (forward, input gradient, weight gradient;
the stem on its pixel-pair view), every BatchNorm forward/backward (single-launch fused
kernels) and the stem's BN-ReLU-max-pool, each timed with HIP events on its launch
stream behind a device sleep (kernel time, not host enqueue time).

For each op: algorithmic FLOPs (real channels) and HBM bytes (each operand read once,
each output written once), average microseconds, achieved TFLOP/s and GB/s, and the
fraction of its own roofline bound = min(MFMA peak, arithmetic intensity x HBM peak)
(peaks: MI355X_MICROARCH.md, 2.5 PFLOP/s dense bf16, 8 TB/s HBM3E).

    python tools/trunk_table.py [--batch 64] [--md out.md] [--reps 10]

Also imported by bench.py (`measure_family`) for the `roofline` object, and run under
`rocprofv3 --pmc` by tools/gpu.sh (pmc_trunk:*) so counters can be attributed per
(kernel, grid) to the same launches.
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MFMA_PEAK_TFS = 2500.0
MFMA_F32_PEAK_TFS = 157.3  # v_mfma_f32_32x32x2_f32 = the f32 vector rate (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0
CL = torch.channels_last

# trunk convolutions of one view (ResNet-18 at 224^2): name, (C, H, W, K, R, stride, pad, count)
TRUNK = [("conv1", (3, 224, 224, 64, 7, 2, 3, 1)), ("l1", (64, 56, 56, 64, 3, 1, 1, 4)),
         ("l2.0.c1", (64, 56, 56, 128, 3, 2, 1, 1)), ("l2.ds", (64, 56, 56, 128, 1, 2, 0, 1)),
         ("l2", (128, 28, 28, 128, 3, 1, 1, 3)), ("l3.0.c1", (128, 28, 28, 256, 3, 2, 1, 1)),
         ("l3.ds", (128, 28, 28, 256, 1, 2, 0, 1)), ("l3", (256, 14, 14, 256, 3, 1, 1, 3)),
         ("l4.0.c1", (256, 14, 14, 512, 3, 2, 1, 1)), ("l4.ds", (256, 14, 14, 512, 1, 2, 0, 1)),
         ("l4", (512, 7, 7, 512, 3, 1, 1, 3))]
# ResNet-50 (Bottleneck, stride on the 3x3 as torchvision v1.5 / resnet.py) of one view at 224^2,
# the C5 workload's trunk: positions with the same shape merged (count per step)
TRUNK50 = [("conv1", (3, 224, 224, 64, 7, 2, 3, 1)),
           ("l1.0.c1", (64, 56, 56, 64, 1, 1, 0, 1)), ("l1.c1", (256, 56, 56, 64, 1, 1, 0, 2)),
           ("l1.c2", (64, 56, 56, 64, 3, 1, 1, 3)), ("l1.c3", (64, 56, 56, 256, 1, 1, 0, 3)),
           ("l1.ds", (64, 56, 56, 256, 1, 1, 0, 1)),
           ("l2.0.c1", (256, 56, 56, 128, 1, 1, 0, 1)), ("l2.0.c2", (128, 56, 56, 128, 3, 2, 1, 1)),
           ("l2.ds", (256, 56, 56, 512, 1, 2, 0, 1)), ("l2.c1", (512, 28, 28, 128, 1, 1, 0, 3)),
           ("l2.c2", (128, 28, 28, 128, 3, 1, 1, 3)), ("l2.c3", (128, 28, 28, 512, 1, 1, 0, 4)),
           ("l3.0.c1", (512, 28, 28, 256, 1, 1, 0, 1)), ("l3.0.c2", (256, 28, 28, 256, 3, 2, 1, 1)),
           ("l3.ds", (512, 28, 28, 1024, 1, 2, 0, 1)), ("l3.c1", (1024, 14, 14, 256, 1, 1, 0, 5)),
           ("l3.c2", (256, 14, 14, 256, 3, 1, 1, 5)), ("l3.c3", (256, 14, 14, 1024, 1, 1, 0, 6)),
           ("l4.0.c1", (1024, 14, 14, 512, 1, 1, 0, 1)), ("l4.0.c2", (512, 14, 14, 512, 3, 2, 1, 1)),
           ("l4.ds", (1024, 14, 14, 2048, 1, 2, 0, 1)), ("l4.c1", (2048, 7, 7, 512, 1, 1, 0, 2)),
           ("l4.c2", (512, 7, 7, 512, 3, 1, 1, 2)), ("l4.c3", (512, 7, 7, 2048, 1, 1, 0, 3))]
TRUNKS = {"resnet18": TRUNK, "resnet50": TRUNK50}
# BatchNorms of one view: name, (C, H, W, residual, relu, count)
BNS = [("bn1", (64, 112, 112, False, True, 1)), ("l1.bn1", (64, 56, 56, False, True, 2)),
       ("l1.bn2", (64, 56, 56, True, True, 2)), ("l2.bn1", (128, 28, 28, False, True, 2)),
       ("l2.bn2", (128, 28, 28, True, True, 2)), ("l2.ds", (128, 28, 28, False, False, 1)),
       ("l3.bn1", (256, 14, 14, False, True, 2)), ("l3.bn2", (256, 14, 14, True, True, 2)),
       ("l3.ds", (256, 14, 14, False, False, 1)), ("l4.bn1", (512, 7, 7, False, True, 2)),
       ("l4.bn2", (512, 7, 7, True, True, 2)), ("l4.ds", (512, 7, 7, False, False, 1))]


def _time(op, reps):
    """Average seconds per call of op() (HIP events on the current stream)."""
    op()
    torch.cuda.synchronize()
    torch.cuda._sleep(20_000_000)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        op()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


def _row(name, op, cnt, flops, nbytes, secs, launches_per_call=1):
    tf = flops / secs / 1e12 if flops else 0.0
    gb = nbytes / secs / 1e9
    bound = min(MFMA_PEAK_TFS, (flops / nbytes) * HBM_PEAK_GBS / 1e3) if flops else None
    frac = (tf / bound) if bound else gb / HBM_PEAK_GBS
    return dict(name=name, op=op, count=cnt, flops=flops, bytes=nbytes, us=secs * 1e6, tflops=tf, gbs=gb,
                bound="mfma" if bound and bound >= MFMA_PEAK_TFS else "hbm", bound_tflops=bound, frac=frac,
                launches=launches_per_call)


def conv_rows(B, dev, reps=10, rotate_bytes=0, dtype="bf16", G=2, arch="resnet18"):
    ops = conv_ops(B, dev, rotate_bytes, G, arch) if dtype == "bf16" else conv_ops_f32(B, dev, rotate_bytes)
    return [_row(name, op, cnt, flops, nbytes, _time(fn, reps)) for name, op, cnt, flops, nbytes, fn in ops]


def _make_f32(op, B, dev, C, H, W, K, R, st, pad, P, Q):
    from greedy_multimodal_learning_amd import conv as G
    from greedy_multimodal_learning_amd import _lib as L
    d = G._desc(B, H, W, C, K, R, R, st, pad)
    x = torch.randn(B, C, H, W, device=dev).contiguous(memory_format=CL)
    w = torch.randn(K, C, R, R, device=dev).contiguous(memory_format=CL)
    dy = torch.randn(B, K, P, Q, device=dev).contiguous(memory_format=CL)
    if op == "fwd":
        y = torch.empty(B, K, P, Q, device=dev).contiguous(memory_format=CL)
        return lambda: G.conv_f32(L.GM_CONV_FWD, d, x=x, w=w, out=y)
    if op == "dgrad":
        dx = torch.empty(B, C, H, W, device=dev).contiguous(memory_format=CL)
        return lambda: G.conv_f32(L.GM_CONV_DGRAD, d, w=w, dy=dy, out=dx)
    dw = torch.empty(K, C, R, R, device=dev).contiguous(memory_format=CL)
    return lambda: G.conv_f32(L.GM_CONV_WGRAD, d, x=x, dy=dy, out=dw)


def conv_ops_f32(B, dev, rotate_bytes=0):
    """The same passes on the reference-precision path: gm_conv2d_f32 (exact-f32 MFMA),
    fp32 channels_last activations, the stem unpadded (what the fp32 drop-in runs)."""
    out = []
    for name, (C, H, W, K, R, st, pad, cnt) in TRUNK:
        P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
        flops = 2.0 * B * P * Q * K * C * R * R
        xb, yb, wb = B * H * W * C * 4, B * P * Q * K * 4, K * C * R * R * 4
        passes = [("fwd", xb + wb + yb), ("wgrad", xb + yb + wb)]
        if C != 3:
            passes.insert(1, ("dgrad", yb + wb + xb))
        for op, nbytes in passes:
            args = (op, B, dev, C, H, W, K, R, st, pad, P, Q)
            sets = max(1, -(-int(rotate_bytes) // nbytes)) if rotate_bytes else 1
            fn = _make_f32(*args) if sets == 1 else _cycle([_make_f32(*args) for _ in range(sets)])
            out.append((name, op, cnt, flops, nbytes, fn))
    return out


def _cycle(fns):
    """One callable that calls fns[0], fns[1], ... in turn (distinct buffer sets)."""
    state = [0]

    def fn():
        f = fns[state[0] % len(fns)]
        state[0] += 1
        return f()
    return fn


def _make_bf16(op, B, dev, C, H, W, K, R, st, pad, P, Q, G=2):
    """A callable running one pass of one trunk convolution position on fresh bf16 operands:
    the G views' launch of the view-batched trunk (vtrunk.py: activations stacked along the
    batch, one weight per view, gm_conv2d_*_grouped_bf16); G = 1 is one view alone."""
    from greedy_multimodal_learning_amd import conv as CV
    from greedy_multimodal_learning_amd import vtrunk as VT
    from greedy_multimodal_learning_amd import _lib as L
    import ctypes
    lib = L.load()
    Cp = CV._cpad(C)
    x = torch.randn(G * B, Cp, H, W, device=dev).bfloat16().contiguous(memory_format=CL)
    dy = torch.randn(G * B, K, P, Q, device=dev).bfloat16().contiguous(memory_format=CL)
    if C == 3:  # the stem runs on the pixel-pair view; its input gradient is never computed
        P_, Q_, Sp, Hp, Wp = CV._stem_geom(H, W, R, R, pad)
        xp = torch.empty(G * B, Hp, Wp // 2, 8, device=dev, dtype=torch.bfloat16)
        wp = torch.empty(G, K, R, Sp, 8, device=dev, dtype=torch.bfloat16)
        for g in range(G):
            CV.stem_pack(x[g * B:(g + 1) * B, :3], torch.randn(K, 3, R, R, device=dev), pad,
                         xp=xp[g * B:(g + 1) * B], wp=wp[g])
        d = CV._desc_hw(B, Hp, Wp // 2, 8, K, R, Sp, 2, 1, 0, 0)
        if op == "fwd":
            y = torch.empty(G * B, K, P, Q, device=dev, dtype=torch.bfloat16)
            return lambda: L.check(lib.gm_conv2d_fwd_grouped_bf16(ctypes.byref(d), G, xp.data_ptr(), wp.data_ptr(),
                                                                  K * R * Sp * 8, y.data_ptr(), 0, 0,
                                                                  L.stream_of(dev)), "stem fwd")
        need = lib.gm_conv2d_wgrad_grouped_scratch(ctypes.byref(d), G)
        scr = torch.empty(max(need, 16), device=dev, dtype=torch.uint8)
        dwp = torch.empty(G, K, R, Sp, 8, device=dev, dtype=torch.float32)
        return lambda: L.check(lib.gm_conv2d_wgrad_grouped_bf16(ctypes.byref(d), G, dy.data_ptr(), xp.data_ptr(),
                                                                dwp.data_ptr(), K * R * Sp * 8, 8, 0, scr.data_ptr(),
                                                                need, L.stream_of(dev)), "stem wgrad")
    n = K * R * R * Cp
    if op == "fwd":
        w = torch.randn(G, K, R, R, Cp, device=dev).bfloat16()
        y = torch.empty(G * B, K, P, Q, device=dev, dtype=torch.bfloat16).contiguous(memory_format=CL)
        d = CV._desc_hw(B, H, W, Cp, K, R, R, st, st, pad, pad)
        ws, nb = VT._splitk_g(dev, CV._desc(B, H, W, Cp, K, R, R, st, pad), G, False)
        return lambda: L.check(lib.gm_conv2d_fwd_grouped_bf16(ctypes.byref(d), G, x.data_ptr(), w.data_ptr(), n,
                                                              y.data_ptr(), ws, nb, L.stream_of(dev)), "fwd")
    if op == "dgrad":
        wt = torch.randn(G, Cp, R, R, K, device=dev).bfloat16()
        dx = torch.empty(G * B, Cp, H, W, device=dev, dtype=torch.bfloat16).contiguous(memory_format=CL)
        d = CV._desc(B, H, W, Cp, K, R, R, st, pad)
        ws, nb = VT._splitk_g(dev, d, G, True)
        return lambda: L.check(lib.gm_conv2d_dgrad_grouped_bf16(ctypes.byref(d), G, dy.data_ptr(), wt.data_ptr(),
                                                                n, dx.data_ptr(), 0, ws, nb, L.stream_of(dev)),
                               "dgrad")
    d = CV._desc_hw(B, H, W, Cp, K, R, R, st, st, pad, pad)
    dw = torch.empty(G, K, R, R, C, device=dev, dtype=torch.float32)
    scr = [torch.empty(16, device=dev, dtype=torch.uint8)]

    def wgrad():  # the scratch the current kernel plan needs (A/B switches change it)
        need = lib.gm_conv2d_wgrad_grouped_scratch(ctypes.byref(d), G)
        if scr[0].numel() < need:
            scr[0] = torch.empty(need, device=dev, dtype=torch.uint8)
        L.check(lib.gm_conv2d_wgrad_grouped_bf16(ctypes.byref(d), G, dy.data_ptr(), x.data_ptr(), dw.data_ptr(),
                                                 K * R * R * C, C, 0, scr[0].data_ptr(), scr[0].numel(),
                                                 L.stream_of(dev)), "wgrad")
    return wgrad


def conv_ops(B, dev, rotate_bytes=0, G=2, arch="resnet18"):
    """(name, pass, count per step, FLOPs, algorithmic bytes, callable) of every trunk
    convolution position at batch B per view, G views per launch (the view-batched trunk).
    rotate_bytes > 0: each callable cycles over enough distinct operand sets that
    consecutive launches touch more than rotate_bytes (beyond the 256 MiB Infinity Cache:
    every launch reads HBM, not the last one's lines)."""
    out = []
    for name, (C, H, W, K, R, st, pad, cnt) in TRUNKS[arch]:
        P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
        flops = 2.0 * G * B * P * Q * K * C * R * R
        xb, yb, wb = G * B * H * W * C * 2, G * B * P * Q * K * 2, G * K * C * R * R * 2
        passes = [("fwd", xb + wb + yb), ("wgrad", xb + yb + G * K * C * R * R * 4)]
        if C != 3:
            passes.insert(1, ("dgrad", yb + wb + xb))
        for op, nbytes in passes:
            args = (op, B, dev, C, H, W, K, R, st, pad, P, Q, G)
            sets = max(1, -(-int(rotate_bytes) // nbytes)) if rotate_bytes else 1
            fn = _make_bf16(*args) if sets == 1 else _cycle([_make_bf16(*args) for _ in range(sets)])
            out.append((name, op, cnt, flops, nbytes, fn))
    return out


def bn_rows(B, dev, reps=10, G=2):
    return [_row(name, op, cnt, flops, nbytes, _time(fn, reps))
            for name, op, cnt, flops, nbytes, fn in bn_ops(B, dev, G)]


def bn_ops(B, dev, G=2):
    """The same for every BatchNorm forward/backward position (the G views' grouped launch,
    gm_bn_*_grouped_bf16) and the stem's statistics + BN-ReLU-max-pool / max-pool backward."""
    import ctypes
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import vtrunk as VT
    lib = L.load()
    out = []
    for name, (C, H, W, res, relu, cnt) in BNS:
        M = B * H * W
        stem = name == "bn1"
        x = torch.randn(G * B, C, H, W, device=dev).bfloat16().contiguous(memory_format=CL)
        r = torch.randn(G * B, C, H, W, device=dev).bfloat16().contiguous(memory_format=CL) if res else None
        dy = torch.randn(G * B, C, H, W, device=dev).bfloat16().contiguous(memory_format=CL)
        y = torch.empty_like(x)
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if res else None
        prm = torch.ones(G, 8, C, device=dev)  # gamma, beta, rm, rv, sm, si, dg, db per view
        prm[:, 1].zero_()
        prm[:, 2].zero_()
        maskx = relu and not res
        coef = torch.empty(G, 2 * C, device=dev)
        buf = VT._bn_scratch_g(dev, M, C, G)
        rows = lambda g: slice(g * B, (g + 1) * B)  # noqa: E731
        fd = [L.BnFwd(M, C, int(relu), x[rows(g)].data_ptr(), r[rows(g)].data_ptr() if res else 0,
                      0 if stem else y[rows(g)].data_ptr(), prm[g, 0].data_ptr(), prm[g, 1].data_ptr(),
                      prm[g, 2].data_ptr(), prm[g, 3].data_ptr(), 0.1, 1e-5, prm[g, 4].data_ptr(), prm[g, 5].data_ptr(),
                      0, coef[g].data_ptr() if maskx else 0) for g in range(G)]
        bd = [L.BnBwd(M, C, int(relu), dy[rows(g)].data_ptr(), 0 if maskx or not relu else y[rows(g)].data_ptr(),
                      x[rows(g)].data_ptr(), prm[g, 0].data_ptr(), prm[g, 4].data_ptr(), prm[g, 5].data_ptr(),
                      dx[rows(g)].data_ptr(), dres[rows(g)].data_ptr() if res else 0, prm[g, 6].data_ptr(),
                      prm[g, 7].data_ptr(), 0, 0, coef[g].data_ptr() if maskx else 0) for g in range(G)]
        fa, ba = L.arr(L.BnFwd, fd), L.arr(L.BnBwd, bd)
        st = L.stream_of(dev)
        fwd_fn = lib.gm_bn_fwd_stats_grouped_bf16 if stem else lib.gm_bn_fwd_train_grouped_bf16

        def fwd(fa=fa, buf=buf, fwd_fn=fwd_fn):
            L.check(fwd_fn(fa, G, buf.data_ptr(), buf.numel(), st), "bn fwd")

        def bwd(ba=ba, buf=buf):
            L.check(lib.gm_bn_bwd_grouped_bf16(ba, G, buf.data_ptr(), buf.numel(), st), "bn bwd")
        fwd()
        e = G * M * C * 2
        out.append((name, "bn_stats" if stem else "bn_fwd", cnt, 0, e * (1 if stem else 2 + (1 if res else 0)), fwd))
        out.append((name, "bn_bwd", cnt, 0, e * (3 + (1 if relu and not maskx else 0) + (1 if res else 0)), bwd))
        if stem:  # the stem's BN + ReLU applied inside the max-pool, and the pool's backward
            P, Q = H // 2, W // 2
            yp = torch.empty(G * B, C, P, Q, device=dev, dtype=torch.bfloat16).contiguous(memory_format=CL)
            idx = torch.empty(G * B, P, Q, C, device=dev, dtype=torch.uint8)
            xs = torch.empty(G * B, P, Q, C, device=dev, dtype=torch.bfloat16)
            gyp = torch.randn(G * B, C, P, Q, device=dev).bfloat16().contiguous(memory_format=CL)
            d1 = L.PoolDesc(B, H, W, C, 3, 2, 1)
            dG = L.PoolDesc(G * B, H, W, C, 3, 2, 1)

            def pool_fwd(d1=d1, x=x, coef=coef, yp=yp, idx=idx, xs=xs):
                L.check(lib.gm_bn_relu_maxpool2d_fwd_grouped_bf16(ctypes.byref(d1), G, x.data_ptr(), coef.data_ptr(),
                                                                  yp.data_ptr(), idx.data_ptr(), xs.data_ptr(), st),
                        "pool fwd")

            def pool_bwd(dG=dG, gyp=gyp, idx=idx, dx=dx):
                L.check(lib.gm_maxpool2d_bwd_bf16(ctypes.byref(dG), gyp.data_ptr(), idx.data_ptr(), dx.data_ptr(),
                                                  st), "pool bwd")
            e_in, e_out = G * M * C, G * B * P * Q * C
            out.append(("maxpool", "bn_relu_fwd", 1, 0, e_in * 2 + e_out * 5, pool_fwd))
            out.append(("maxpool", "bwd", 1, 0, e_out * 3 + e_in * 2, pool_bwd))
            pool_fwd()  # valid argmax bytes for the fused backward

            def pool_bn_bwd(d1=d1, gyp=gyp, idx=idx, xs=xs, ba=ba, buf=buf):  # what the step runs (vtrunk)
                L.check(lib.gm_bn_relu_maxpool2d_bwd_grouped_bf16(ctypes.byref(d1), G, gyp.data_ptr(), idx.data_ptr(),
                                                                  xs.data_ptr(), ba, buf.data_ptr(), buf.numel(), st),
                        "pool+bn bwd")
            # pass 1: pooled gradient + selected x; pass 2: x, pooled gradient, argmax, the dx write
            out.append(("bn1+maxpool", "pool_bn_bwd", 1, 0, e_out * 4 + (e_in * 2 + e_out * 3) + e_in * 2, pool_bn_bwd))
    return out


def measure_family(B, dev, reps=10, rotate_bytes=320e6, dtype="bf16", G=2, arch="resnet18"):
    """The conv family (fwd + dgrad + wgrad of every trunk position, weighted by its count
    per step; bf16: the G views' grouped launches the step runs, fp32: one view's launches,
    the reference-precision path runs the views one by one): (flops, secs, launches, rows).
    Launches rotate over operand sets of more than the 256 MiB Infinity Cache
    (rotate_bytes), so none reads warm lines."""
    rows = conv_rows(B, dev, reps, rotate_bytes, dtype, G, arch)
    flops = sum(r["flops"] * r["count"] for r in rows)
    secs = sum(r["us"] * 1e-6 * r["count"] for r in rows)
    launches = sum(r["count"] for r in rows)
    return flops, secs, launches, rows


def markdown(rows, B, G=2, arch="resnet18"):
    out = [f"{arch}: {G} view(s) per launch ({'view-batched trunk' if G > 1 else 'per-view launches'}), "
           f"batch {B} per view", "",
           f"| shape | pass | x/step | GFLOP | MB | avg us | TFLOP/s | GB/s | bound | frac of bound |",
           "|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        bt = f"mfma {MFMA_PEAK_TFS:.0f}" if r["bound"] == "mfma" and r["flops"] else (
            f"AIxHBM {r['bound_tflops']:.0f} TF" if r["flops"] else "hbm 8000 GB/s")
        out.append(f"| {r['name']} | {r['op']} | {r['count']} | {r['flops'] / 1e9:.2f} | {r['bytes'] / 1e6:.1f} | "
                   f"{r['us']:.1f} | {r['tflops']:.1f} | {r['gbs']:.0f} | {bt} | {r['frac']:.3f} |")
    cf = [r for r in rows if r["flops"]]
    fl = sum(r["flops"] * r["count"] for r in cf)
    s = sum(r["us"] * r["count"] for r in cf) * 1e-6
    out.append("")
    if cf:
        out.append(f"conv family ({G} view(s) per launch, B={B} per view): {fl / 1e12:.3f} TFLOP in {s * 1e3:.3f} ms = "
                   f"{fl / s / 1e12:.1f} TFLOP/s = {fl / s / 1e12 / MFMA_PEAK_TFS:.3f} of {MFMA_PEAK_TFS:.0f} TF")
    hb = [r for r in rows if not r["flops"]]
    if hb:
        by = sum(r["bytes"] * r["count"] for r in hb)
        s2 = sum(r["us"] * r["count"] for r in hb) * 1e-6
        out.append(f"BN + max-pool ({G} view(s) per launch): {by / 1e9:.3f} GB in {s2 * 1e3:.3f} ms = {by / s2 / 1e9:.0f} GB/s "
                   f"= {by / s2 / 1e9 / HBM_PEAK_GBS:.3f} of {HBM_PEAK_GBS:.0f} GB/s")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--groups", type=int, default=2, help="views per launch (2: the step's view-batched trunk)")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--md", default=None)
    ap.add_argument("--only", default="", help="conv | bn (default both)")
    ap.add_argument("--arch", default="resnet18", choices=sorted(TRUNKS),
                    help="trunk (resnet50: the C5 workload's, convolutions only; use --groups 1 --batch 32)")
    ap.add_argument("--rotate-mb", type=float, default=320.0,
                    help="conv launches rotate over operand sets of this many MB (0: one warm set)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from greedy_multimodal_learning_amd import build
    build.build()
    rows = []
    if a.only in ("", "conv"):
        rows += conv_rows(a.batch, dev, a.reps, a.rotate_mb * 1e6, G=a.groups, arch=a.arch)
    if a.only in ("", "bn") and a.arch == "resnet18":
        rows += bn_rows(a.batch, dev, a.reps, a.groups)
    md = markdown(rows, a.batch, a.groups, a.arch)
    print(md)
    if a.md:
        with open(a.md, "w") as f:
            f.write(md + "\n")


if __name__ == "__main__":
    main()
