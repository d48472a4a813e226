"""View-batched trunk: the G unshared ResNet trunks of the multi-view model as ONE stacked trunk.

The reference runs its two view trunks one after the other (src/model.py:65-106: `net_view_0`
then `net_view_1`, torchvision resnet18 pieces, MMTM after layer2/3/4).  The trunks have
identical shapes and different weights, so on MI355X every convolution / BatchNorm of a
block position is ONE launch over both views: the activations are stacked along the batch
([G*B, C, H, W] channels_last bf16, view g = rows g*B .. (g+1)*B-1) and each kernel takes
the G weights (or the G parameter / statistic sets) of that position:

    conv fwd / dgrad : gm_conv2d_{fwd,dgrad}_grouped_bf16 (weight g at wb + g*stride)
    conv wgrad       : gm_conv2d_wgrad_grouped_bf16 (dW g at grad + g*stride: the engine's
                       flat gradient buffer lays the views' parameters out at one stride)
    BatchNorm        : gm_bn_{fwd_train,bwd,fwd_stats}_grouped_bf16 (per-view statistics,
                       running stats, num_batches_tracked: exactly the per-view modules')
    stem pool        : gm_bn_relu_maxpool2d_fwd_grouped_bf16

Layer 3/4 grids of one view (B = 64: 49-196 output tiles) leave most of the 256 CUs idle;
stacked, the launch count halves and each grid doubles.  The arithmetic per view is the
per-view trunk's (same kernels, same tile order within a view): the stacked trunk is
checked against the per-view trunk in tests/test_gpu_vtrunk.py.

The modules stay what they are (`net_view_i.layer*.conv*` / `bn*` parameters, buffers,
state_dict); this executor only reads them.  Training-mode bf16 only; everything else
takes the per-view path (model.MMTM_MVCNN.forward decides).
"""
import contextlib
import ctypes
import os

import torch

from .streams import zeroed_scratch
from . import _lib as L
from .bn import MASK_FROM_X
from .conv import CL, _cpad, _desc, _desc_hw, _like_param, _prepped, _splitk_ws, _stem_geom, stem_pack, \
    stem_pack_grouped
from .gradsink import GradJoin, MaskedAddend, sink_done, sink_pending, sink_target

BF = torch.bfloat16
ENABLED = os.environ.get("GM_VTRUNK", "1") != "0"


# the stem's pool + BN backward in the gathered two-pass form (False: the max-pool backward +
# BatchNorm backward pair; module switches below are A/B and test switches)
FUSED_STEM_BWD = True
# its statistics pass over the pooled tensors (the forward's selected x) instead of x
STEM_XSEL = True
# with it, the stem's weight gradient forms its dy in the loader from the pool + BN operands, so
# the BN's input gradient (the stem's dy, 205 MB at C2) is never written nor read (False: the
# BN backward's apply pass writes it, the weight gradient reads it)
FUSED_STEM_WGRAD = True
# the stem BN's statistics from the stem convolution's epilogue (False: the statistics pass over
# the convolution's output)
FUSED_STEM_STATS = True
# every other BatchNorm's statistics from its producing convolution's epilogue, then a finalize
# and a streaming apply instead of the single-launch BatchNorm's statistics read
# (False: the single-launch BatchNorm)
EPI_BN_STATS = True
# the block-output BatchNorm (+ residual + ReLU) writes its ReLU mask as bits (1/16 of y) and the
# backward reads them in place of y (False: the backward reads y)
BN_RELU_MASK = True
# with it, a downsample block's residual BN backward reads the block output BN's dy and ReLU mask
# (the fused backward's mask mode) instead of the dres = dz tensor that BN would otherwise write
DS_DZ_LINK = True
# and an identity block's: the block input's gradient join hands conv1's dgrad the pending addend as
# (dy, mask) (gradsink.MaskedAddend; gm_conv2d_dgrad_grouped_masked_bf16) - no dres either
IDT_MASKED_ADDEND = True
# the ReLU-after-BN backward (bn1 / bn2 of a block) takes its statistics from the input-gradient
# epilogue of the convolution it feeds, then one finalize + one streaming apply
# (False: the single-launch backward)
EPI_BN_BWD_STATS = True
_GM_E_UNSUP = -3


def _nhwc(t):
    return t if t.is_contiguous(memory_format=CL) else t.contiguous(memory_format=CL)


def _stride(ts, elem_bytes):
    """Element stride between consecutive tensors' storage if it is one constant (0 for a
    single tensor; negative when the later views sit lower, as in the engine's flat buffer,
    which is laid out in reverse registration order), else None."""
    if len(ts) < 2:
        return 0
    d = ts[1].data_ptr() - ts[0].data_ptr()
    if d == 0 or d % elem_bytes:
        return None
    for a, b in zip(ts[1:], ts[2:]):
        if b.data_ptr() - a.data_ptr() != d:
            return None
    return d // elem_bytes


def _splitk_g(device, d, G, dgrad):
    """Split-K workspace (shared with the per-view convolutions: its turnstile words sit in
    a fixed region, so one zeroed buffer per stream serves both)."""
    need = L.load().gm_conv2d_splitk_ws_bytes_grouped(ctypes.byref(d), G, int(dgrad))
    if need == 0:
        return 0, 0
    buf = zeroed_scratch(_splitk_ws, device, need, lambda old: (need + (1 << 20) - 1) >> 20 << 20)
    return buf.data_ptr(), buf.numel()


_bn_scratch = {}


def _bn_scratch_g(device, M, C, G):
    """Grouped-layout BatchNorm scratch per (device, stream), zeroed once (its ticket words
    sit in fixed per-group headers: never shared with the ungrouped calls' buffers)."""
    need = L.load().gm_bn_scratch_grouped(M, C, G)
    return zeroed_scratch(_bn_scratch, device, need,
                          lambda old: max(need, 1 << 20) if old is None else max(need, 2 * old.numel()))


@L.on_fault_reset
def _reset_bn_scratch():
    for buf in _bn_scratch.values():
        buf.zero_()
    torch.cuda.synchronize()


# ---- convolution -------------------------------------------------------------------

WGRAD_STREAM = True
_WGRAD_SIDE = 64  # streams.side_stream index of the weight-gradient stream
# Weight-gradient launches are handed to the wgrad stream in batches of WGRAD_BATCH (one
# stream fork per batch; 1 = a fork per convolution).  In a replayed
# hipGraph every fork makes the main chain's next node start on another hardware queue,
# ~15-25 us of idle GPU per hop (profiles/r03e_step_listing.txt, tools/trace_gaps.py).
# A batch is flushed when full, by the stem's backward (the trunk's last), and at the end
# of the backward pass (autograd queue_callback), so no launch is ever left pending.
WGRAD_BATCH = 8
_PENDING = []  # (launch, weights, tensors to keep alive, device)


def flush_wgrads():
    """Launch the pending weight gradients on the wgrad stream (one fork) and report their
    parameters' gradients delivered (gradsink)."""
    if not _PENDING:
        return
    items = list(_PENDING)
    _PENDING.clear()
    dev = items[0][3]
    side = _wgrad_stream(dev)
    if side is not None:
        side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
        for launch, _, keep, _ in items:
            if side is not None:
                for t in keep:
                    t.record_stream(side)
            launch()
    for _, weights, _, _ in items:
        for w in weights:
            sink_done(w)


def drop_pending_wgrads():
    """Forget weight-gradient launches a failed backward left queued (the autograd
    end-of-backward callback does not run when backward raises).  Called by the engine
    at the start of every step and on its error path, so a stale closure (old gy / x,
    possibly capture-pool memory) is never launched into the next step's gradients."""
    n = len(_PENDING)
    _PENDING.clear()
    return n


def _defer_wgrad(launch, weights, keep, dev):
    for w in weights:
        sink_pending(w)
    if not _PENDING:
        torch.autograd.Variable._execution_engine.queue_callback(flush_wgrads)
    _PENDING.append((launch, weights, keep, dev))
    if len(_PENDING) >= WGRAD_BATCH:
        flush_wgrads()


def _wgrad_stream(dev):
    if not WGRAD_STREAM or dev.type != "cuda":
        return None
    from .streams import side_stream
    return side_stream(dev, _WGRAD_SIDE)


def _group_weights(weights, Cp, need_t):
    """bf16 KRSC copies of the G weights at one stride: the step's WeightPrep copies when
    they are laid out that way (the engine's), else a fresh stacked prep.  Returns
    (wb, wb_stride, wt, wt_stride) with wb / wt the group-0 tensors."""
    pre = [_prepped.get(w.data_ptr()) for w in weights] if _prepped else [None]
    if all(p is not None and (p[1] is not None or not need_t) for p in pre):
        wbs, wts = [p[0] for p in pre], [p[1] for p in pre]
        sb = _stride(wbs, 2)
        st = _stride(wts, 2) if need_t else 0
        n = wbs[0].numel()
        if sb is not None and st is not None and (len(wbs) == 1 or (abs(sb) >= n and (not need_t or abs(st) >= n))):
            return wbs[0], sb, wts[0], st
    lib = L.load()
    G = len(weights)
    K, C, R, S = weights[0].shape
    dev = weights[0].device
    wb = torch.empty(G, K, R, S, Cp, device=dev, dtype=BF)
    wt = torch.empty(G, Cp, R, S, K, device=dev, dtype=BF) if need_t else None
    for g, w in enumerate(weights):
        w32 = _nhwc(w.detach().float())
        L.check(lib.gm_conv_weight_prep_bf16(w32.data_ptr(), K, R * S, C, Cp, wb[g].data_ptr(),
                                             wt[g].data_ptr() if need_t else 0, L.stream_of(dev)),
                "gm_conv_weight_prep_bf16")
    n = K * R * S * Cp
    return wb[0], n, (wt[0] if need_t else None), n


class _VConvFn(torch.autograd.Function):
    """y = conv(X_g, W_g) for every view group g of the stacked X, one launch per pass."""

    @staticmethod
    def forward(ctx, X, G, stride, pad, join, stats, *weights):
        """stats (optional dict): receives the BatchNorm statistics partial rows of the output
        from the epilogue (gm_conv2d_fwd_grouped_bn_stats_bf16) when the kernel has them."""
        lib = L.load()
        ctx.join = join
        # the BatchNorm that produced X (vblock: bn1 -> relu -> conv2), for its backward
        # statistics from this convolution's input-gradient epilogue
        ctx.dlink = stats.get("dgrad_link") if stats is not None else None
        GN, C, H, W = X.shape
        N = GN // G
        K, C0, R, S = weights[0].shape
        if C != C0 or _cpad(C) != C or GN != N * G:
            raise L.GreedyMMLError(f"vtrunk conv: stacked input {tuple(X.shape)} does not fit {G} x {C0} channels")
        xb = _nhwc(X.to(BF))
        need_dx = ctx.needs_input_grad[0]
        wb, sb, wt, st = _group_weights(weights, C, need_dx)
        P = (H + 2 * pad - R) // stride + 1
        Q = (W + 2 * pad - S) // stride + 1
        y = torch.empty(GN, K, P, Q, device=X.device, dtype=BF, memory_format=CL)
        d = _desc_hw(N, H, W, C, K, R, S, stride, stride, pad, pad)
        ws, nb = _splitk_g(X.device, _desc(N, H, W, C, K, R, S, stride, pad), G, False)
        rc = _GM_E_UNSUP
        if stats is not None and EPI_BN_STATS and K % 64 == 0:
            nf = lib.gm_conv2d_fwd_bn_stats_floats(ctypes.byref(d), G)
            part = torch.empty(max(nf, 1), device=X.device, dtype=torch.float32)
            rows = ctypes.c_int(0)
            rc = lib.gm_conv2d_fwd_grouped_bn_stats_bf16(ctypes.byref(d), G, xb.data_ptr(), wb.data_ptr(), sb,
                                                         y.data_ptr(), part.data_ptr(), nf, ctypes.byref(rows), ws,
                                                         nb, L.stream_of(X.device))
            if rc == 0:
                stats["part"], stats["rows"] = part, rows.value
            elif rc != _GM_E_UNSUP:
                L.check(rc, "gm_conv2d_fwd_grouped_bn_stats_bf16")
        if rc != 0:
            L.check(lib.gm_conv2d_fwd_grouped_bf16(ctypes.byref(d), G, xb.data_ptr(), wb.data_ptr(), sb, y.data_ptr(),
                                                   ws, nb, L.stream_of(X.device)), "gm_conv2d_fwd_grouped_bf16")
        ctx.save_for_backward(xb, wt, *weights)
        ctx.meta = (G, N, stride, pad, st)
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = L.load()
        xb, wt, *weights = ctx.saved_tensors
        G, N, stride, pad, st = ctx.meta
        GN, C, H, W = xb.shape
        K, _, R, S = weights[0].shape
        gy = _nhwc(gy.to(BF))
        dev = gy.device
        dx = None
        if ctx.needs_input_grad[0]:
            d = _desc(N, H, W, C, K, R, S, stride, pad)

            def dgrad(add):
                madd = add if isinstance(add, MaskedAddend) else None
                at = madd.dy if madd is not None else add
                if at is not None and (tuple(at.shape) != (GN, C, H, W) or at.dtype != BF
                                       or not at.is_contiguous(memory_format=CL)):
                    raise ValueError("vtrunk conv dgrad: addend must be bf16 channels_last shaped like dx")
                if madd is not None:  # dx = dgrad + dy where the block output's ReLU passed
                    if madd.mask.numel() * 8 != at.numel():
                        raise ValueError("vtrunk conv dgrad: addend mask must hold one bit per element")
                    out = torch.empty(GN, C, H, W, device=dev, dtype=BF, memory_format=CL)
                    ws, nb = _splitk_g(dev, d, G, True)
                    L.check(lib.gm_conv2d_dgrad_grouped_masked_bf16(
                        ctypes.byref(d), G, gy.data_ptr(), wt.data_ptr(), st, out.data_ptr(), at.data_ptr(),
                        madd.mask.data_ptr(), ws, nb, L.stream_of(dev)), "gm_conv2d_dgrad_grouped_masked_bf16")
                    return out
                out = add if add is not None else torch.empty(GN, C, H, W, device=dev, dtype=BF, memory_format=CL)
                ws, nb = _splitk_g(dev, d, G, True)
                lk = ctx.dlink
                if add is None and lk is not None and "bn" in lk and EPI_BN_BWD_STATS:
                    bx, bcoef, bmean = lk.pop("bn")
                    if tuple(bx.shape) == (GN, C, H, W):
                        nf = lib.gm_conv2d_dgrad_bn_stats_floats(ctypes.byref(d), G)
                        part = torch.empty(max(nf, 1), device=dev, dtype=torch.float32)
                        rows = ctypes.c_int(0)
                        rc = lib.gm_conv2d_dgrad_grouped_bn_stats_bf16(
                            ctypes.byref(d), G, gy.data_ptr(), wt.data_ptr(), st, out.data_ptr(), bx.data_ptr(),
                            bcoef.data_ptr(), bmean.data_ptr(), part.data_ptr(), nf, ctypes.byref(rows), ws, nb,
                            L.stream_of(dev))
                        if rc == 0:
                            lk["part"], lk["rows"], lk["dy"] = part, rows.value, out
                            return out
                        if rc != _GM_E_UNSUP:
                            L.check(rc, "gm_conv2d_dgrad_grouped_bn_stats_bf16")
                L.check(lib.gm_conv2d_dgrad_grouped_bf16(ctypes.byref(d), G, gy.data_ptr(), wt.data_ptr(), st,
                                                         out.data_ptr(), L.ptr(add), ws, nb, L.stream_of(dev)),
                        "gm_conv2d_dgrad_grouped_bf16")
                return out
            dx = ctx.join.contribute(dgrad) if ctx.join is not None else dgrad(None)
        grads = [None] * G
        want = [ctx.needs_input_grad[6 + g] for g in range(G)]
        if any(want):
            dh = _desc_hw(N, H, W, C, K, R, S, stride, stride, pad, pad)
            tg = [sink_target(w) if wn else None for w, wn in zip(weights, want)]
            need = lib.gm_conv2d_wgrad_grouped_scratch(ctypes.byref(dh), G)
            scratch = torch.empty(max(need, 16), device=dev, dtype=torch.uint8)
            sunk = all(t is not None for t in tg)
            if sunk:
                bufs = [t[0] for t in tg]
                sd = _stride(bufs, 4)
                if (sd is None or len({t[1] for t in tg}) != 1 or (G > 1 and abs(sd) < bufs[0].numel())
                        or not all(b.is_contiguous(memory_format=CL) for b in bufs)):
                    raise RuntimeError("vtrunk conv: the views' gradient buffers must be channels_last, one "
                                       "accumulate state, at one stride (the engine's flat layout)")
                # the weight gradient is off the critical path (only the step's end reads it):
                # it runs on the wgrad stream, overlapping the next input-gradient launches;
                # the engine joins the side streams before the gradients are read
                def launch(dh=dh, gy=gy, xb=xb, buf=bufs[0], sd=sd, acc=int(tg[0][1]), scratch=scratch, need=need):
                    L.check(lib.gm_conv2d_wgrad_grouped_bf16(ctypes.byref(dh), G, gy.data_ptr(), xb.data_ptr(),
                                                             buf.data_ptr(), sd, C, acc, scratch.data_ptr(), need,
                                                             L.stream_of(dev)), "gm_conv2d_wgrad_grouped_bf16")
                if _wgrad_stream(dev) is not None:
                    _defer_wgrad(launch, list(weights), (gy, xb, scratch), dev)
                else:
                    launch()
                    for w in weights:
                        sink_done(w)
            else:
                if any(t is not None for t in tg):
                    raise RuntimeError("vtrunk conv: all or none of the views' weights must be sink-managed")
                dw = torch.empty(G, K, R, S, C, device=dev, dtype=torch.float32)
                L.check(lib.gm_conv2d_wgrad_grouped_bf16(ctypes.byref(dh), G, gy.data_ptr(), xb.data_ptr(),
                                                         dw.data_ptr(), K * R * S * C, C, 0, scratch.data_ptr(),
                                                         need, L.stream_of(dev)), "gm_conv2d_wgrad_grouped_bf16")
                grads = [_like_param(dw[g].permute(0, 3, 1, 2), w) if wn else None
                         for g, (w, wn) in enumerate(zip(weights, want))]
        return (dx, None, None, None, None, None, *grads)


def vconv(X, convs, join=None, stats=None):
    """The G GMConv2d modules `convs` (one per view, same shape) over the stacked X; `stats`
    (a dict) receives the output's BatchNorm partial rows for vbn(..., stats=) when the
    convolution's kernel produces them."""
    c0 = convs[0]
    if not c0._hip_ok():
        raise L.GreedyMMLError("vtrunk conv: only the ResNet trunk's convolutions")
    if join is not None and X.requires_grad and torch.is_grad_enabled():
        join.register()
    else:
        join = None
    with torch.autocast("cuda", enabled=False):
        return _VConvFn.apply(X, len(convs), c0.stride[0], c0.padding[0], join, stats, *[c.weight for c in convs])


# ---- BatchNorm ---------------------------------------------------------------------

def _bn_param_grads(gammas, betas, want_w, want_b):
    """Per-view (dgamma, dbeta) buffers: the sink targets when the engine armed them (one
    accumulate state for all views), else fresh.  Returns (dgs, dbs, acc, sunk)."""
    G = len(gammas)
    tw = [sink_target(w) for w in gammas] if want_w and want_b else []
    tb = [sink_target(b) for b in betas] if want_w and want_b else []
    if tw and all(t is not None for t in tw + tb):
        accs = {t[1] for t in tw + tb}
        if len(accs) != 1:
            raise RuntimeError("vtrunk BatchNorm: the views' parameters must share one gradient sink state")
        return [t[0] for t in tw], [t[0] for t in tb], accs.pop(), True
    if any(t is not None for t in tw + tb):
        raise RuntimeError("vtrunk BatchNorm: all or none of the views' parameters must be sink-managed")
    C = gammas[0].shape[0]
    dev = gammas[0].device
    return ([torch.empty(C, device=dev, dtype=torch.float32) for _ in range(G)],
            [torch.empty(C, device=dev, dtype=torch.float32) for _ in range(G)], False, False)


def _bn_backward(dz, y, xb, G, gammas, betas, sm, si, relu, want_dres, coef, want_w, want_b, ymask=None):
    """Grouped BN backward; returns (dx, dres, grads_w[G], grads_b[G]).  ymask: the forward's
    ReLU mask bytes (read in place of y by the single-launch backward)."""
    lib = L.load()
    GN, C, H, W = xb.shape
    M = (GN // G) * H * W
    dz = _nhwc(dz.to(BF))
    dx = torch.empty_like(xb, memory_format=CL)
    dres = torch.empty_like(xb, memory_format=CL) if want_dres else None
    dgs, dbs, acc, sunk = _bn_param_grads(gammas, betas, want_w, want_b)
    descs = []
    for g in range(G):
        r = slice(g * (GN // G), (g + 1) * (GN // G))
        descs.append(L.BnBwd(M, C, int(relu), dz[r].data_ptr(), y[r].data_ptr() if (relu and y is not None) else 0,
                             xb[r].data_ptr(), gammas[g].data_ptr(), sm[g].data_ptr(), si[g].data_ptr(),
                             dx[r].data_ptr(), dres[r].data_ptr() if dres is not None else 0, dgs[g].data_ptr(),
                             dbs[g].data_ptr(), int(acc), 0, coef[g].data_ptr() if coef is not None else 0,
                             ymask[g * (M * C // 8):].data_ptr() if ymask is not None else 0))
    buf = _bn_scratch_g(xb.device, M, C, G)
    L.check(lib.gm_bn_bwd_grouped_bf16(L.arr(L.BnBwd, descs), G, buf.data_ptr(), buf.numel(),
                                       L.stream_of(xb.device)), "gm_bn_bwd_grouped_bf16")
    if sunk:
        for p in list(gammas) + list(betas):
            sink_done(p)
        return dx, dres, [None] * G, [None] * G
    return dx, dres, [d if want_w else None for d in dgs], [d if want_b else None for d in dbs]


def _bn_backward_from_stats(dz, xb, G, gammas, betas, sm, si, coef, part, rows, want_w, want_b):
    """The ReLU-after-BN backward with its statistics from the input-gradient epilogue of the
    convolution that consumed the BN's output (gm_conv2d_dgrad_grouped_bn_stats_bf16): an fp64
    finalize and one streaming apply.  Returns (dx, grads_w[G], grads_b[G])."""
    lib = L.load()
    GN, C, H, W = xb.shape
    M = (GN // G) * H * W
    dx = torch.empty_like(xb, memory_format=CL)
    dgs, dbs, acc, sunk = _bn_param_grads(gammas, betas, want_w, want_b)
    descs = []
    for g in range(G):
        r = slice(g * (GN // G), (g + 1) * (GN // G))
        descs.append(L.BnBwd(M, C, 1, dz[r].data_ptr(), 0, xb[r].data_ptr(), gammas[g].data_ptr(),
                             sm[g].data_ptr(), si[g].data_ptr(), dx[r].data_ptr(), 0, dgs[g].data_ptr(),
                             dbs[g].data_ptr(), int(acc), 0, coef[g].data_ptr(), 0))
    st = L.stream_of(xb.device)
    arr = L.arr(L.BnBwd, descs)
    L.check(lib.gm_bn_bwd_stats_finalize_grouped(arr, G, part.data_ptr(), rows, st), "gm_bn_bwd_stats_finalize_grouped")
    L.check(lib.gm_bn_bwd_apply_grouped_bf16(arr, G, part.data_ptr(), rows, st), "gm_bn_bwd_apply_grouped_bf16")
    if sunk:
        for p in list(gammas) + list(betas):
            sink_done(p)
        return dx, [None] * G, [None] * G
    return dx, [d if want_w else None for d in dgs], [d if want_b else None for d in dbs]


class _VBNFn(torch.autograd.Function):
    """relu?(BatchNorm_g(X_g) (+ residual_g)) per view group g of the stacked X."""

    @staticmethod
    def forward(ctx, X, residual, G, bns, relu, join, stats, *params):
        lib = L.load()
        ctx.join = join
        gammas, betas = params[:G], params[G:]
        xb = _nhwc(X.to(BF))
        GN, C, H, W = xb.shape
        N = GN // G
        M = N * H * W
        if residual is not None:
            residual = _nhwc(residual.to(BF))
        maskx = relu and residual is None and MASK_FROM_X
        y = torch.empty_like(xb, memory_format=CL)
        dev = xb.device
        sm = torch.empty(G, C, device=dev, dtype=torch.float32)
        si = torch.empty(G, C, device=dev, dtype=torch.float32)
        coef = torch.empty(G, 2 * C, device=dev, dtype=torch.float32) if maskx else None
        ymask = (torch.empty(GN * H * W * C // 8, device=dev, dtype=torch.uint8)
                 if relu and residual is not None and BN_RELU_MASK else None)
        descs = []
        for g, bn in enumerate(bns):
            r = slice(g * N, (g + 1) * N)
            descs.append(L.BnFwd(M, C, int(relu), xb[r].data_ptr(),
                                 residual[r].data_ptr() if residual is not None else 0, y[r].data_ptr(),
                                 gammas[g].data_ptr(), betas[g].data_ptr(), L.ptr(bn.running_mean),
                                 L.ptr(bn.running_var), float(bn.momentum), float(bn.eps), sm[g].data_ptr(),
                                 si[g].data_ptr(), L.ptr(bn.num_batches_tracked),
                                 coef[g].data_ptr() if maskx else 0,
                                 ymask[g * (M * C // 8):].data_ptr() if ymask is not None else 0))
        if stats is not None and "part" in stats:  # partial rows from the convolution's epilogue
            part, rows = stats.pop("part"), stats.pop("rows")
            st = L.stream_of(dev)
            L.check(lib.gm_bn_fwd_stats_finalize_grouped(L.arr(L.BnFwd, descs), G, part.data_ptr(), rows, st),
                    "gm_bn_fwd_stats_finalize_grouped")
            L.check(lib.gm_bn_fwd_apply_grouped_bf16(L.arr(L.BnFwd, descs), G, part.data_ptr(), rows, st),
                    "gm_bn_fwd_apply_grouped_bf16")
        else:
            buf = _bn_scratch_g(dev, M, C, G)
            L.check(lib.gm_bn_fwd_train_grouped_bf16(L.arr(L.BnFwd, descs), G, buf.data_ptr(), buf.numel(),
                                                     L.stream_of(dev)), "gm_bn_fwd_train_grouped_bf16")
        ctx.save_for_backward(xb, y if relu and not maskx else coef, sm, si, ymask, *gammas, *betas)
        ctx.meta = (G, maskx, relu, residual is not None)
        ctx.blink = stats.get("bn_link") if stats is not None else None
        # res_link (block output BN): the residual's BN backward takes this BN's dy and ReLU
        # mask instead of a materialised dres; dz_link (that residual BN): where it finds them
        ctx.rlink = stats.get("res_link") if stats is not None and ymask is not None else None
        ctx.zlink = stats.get("dz_link") if stats is not None and not relu and residual is None else None
        if ctx.blink is not None and maskx and G >= 2 and C % 64 == 0:
            ctx.blink["bn"] = (xb, coef, sm)  # for the consuming convolution's input-gradient epilogue
        return y

    @staticmethod
    def backward(ctx, dy):
        xb, yc, sm, si, ymask, *prm = ctx.saved_tensors
        G, maskx, relu, has_res = ctx.meta
        gammas, betas = prm[:G], prm[G:]
        y, coef = (None, yc) if maskx else (yc, None)
        want_dres = has_res and ctx.needs_input_grad[1]
        lk = ctx.blink
        want_w, want_b = any(ctx.needs_input_grad[7:7 + G]), any(ctx.needs_input_grad[7 + G:])
        if lk is not None and "part" in lk:  # statistics from the consuming convolution's dgrad
            part, rows, pdy = lk.pop("part"), lk.pop("rows"), lk.pop("dy")
            lk.pop("bn", None)
            if maskx and not want_dres and dy.data_ptr() == pdy.data_ptr() and dy.shape == pdy.shape:
                dx, gw, gb = _bn_backward_from_stats(pdy, xb, G, gammas, betas, sm, si, coef, part, rows,
                                                     want_w, want_b)
                return (dx if ctx.needs_input_grad[0] else None, None, None, None, None, None, None, *gw, *gb)
        zl = ctx.zlink
        if zl is not None and "dz" in zl:  # dy is the block output's: dz = dy where its ReLU passed
            dyo, yo, mo = zl.pop("dz")
            if dy.data_ptr() != dyo.data_ptr() or dy.shape != dyo.shape:
                raise L.GreedyMMLError("vtrunk BatchNorm: the residual's gradient is not the block output's dy")
            dx, _, gw, gb = _bn_backward(dyo, yo, xb, G, gammas, betas, sm, si, True, False, None,
                                         want_w, want_b, mo)
            return (dx if ctx.needs_input_grad[0] else None, None, None, None, None, None, None, *gw, *gb)
        join = ctx.join
        if (want_dres and join is not None and ymask is not None and IDT_MASKED_ADDEND and join.masked_ok
                and join.first_of_many()):
            # the identity branch: the block input's other consumer (conv1) forms dz = dy . mask
            # in its dgrad epilogue; no dres written here
            dyb = _nhwc(dy.to(BF))
            dx, _, gw, gb = _bn_backward(dyb, y, xb, G, gammas, betas, sm, si, relu, False, coef,
                                         want_w, want_b, ymask)
            join.contribute(lambda add: MaskedAddend(dyb, ymask))
            return (dx if ctx.needs_input_grad[0] else None, None, None, None, None, None, None, *gw, *gb)
        if want_dres and ctx.rlink is not None and DS_DZ_LINK:
            dyb = _nhwc(dy.to(BF))
            ctx.rlink["dz"] = (dyb, y, ymask)
            dx, _, gw, gb = _bn_backward(dyb, y, xb, G, gammas, betas, sm, si, relu, False, coef,
                                         want_w, want_b, ymask)
            return (dx if ctx.needs_input_grad[0] else None, dyb, None, None, None, None, None, *gw, *gb)
        dx, dres, gw, gb = _bn_backward(dy, y, xb, G, gammas, betas, sm, si, relu, want_dres, coef,
                                        want_w, want_b, ymask)
        if dres is not None and ctx.join is not None:
            dres = ctx.join.contribute(lambda add: dres if add is None else dres + add)
        return (dx if ctx.needs_input_grad[0] else None, dres, None, None, None, None, None, *gw, *gb)


def vbn(X, bns, residual=None, relu=False, residual_join=None, stats=None):
    """The G GMBatchNorm2d modules `bns` (training mode) over the stacked X."""
    b0 = bns[0]
    if any(b.momentum is None or b.momentum != b0.momentum or b.eps != b0.eps for b in bns):
        raise L.GreedyMMLError("vtrunk BatchNorm: the views must share momentum and eps")
    join = None
    if residual_join is not None and residual is not None and residual.requires_grad and torch.is_grad_enabled():
        residual_join.register()
        join = residual_join
    with torch.autocast("cuda", enabled=False):
        return _VBNFn.apply(X, residual, len(bns), bns, bool(relu), join, stats,
                            *[b.weight for b in bns], *[b.bias for b in bns])


# ---- stem: 7x7/s2 convolution on the pixel-pair view, BN + ReLU + max-pool --------------

class _VStemFn(torch.autograd.Function):
    """The G views' RGB stems: view g = x[:, g] (the model input [B, G, C0, H, W]),
    packed into one stacked pair view and convolved in one launch."""

    @staticmethod
    def forward(ctx, x, G, pad, stats, *weights):
        """stats (optional dict): receives the BN statistics partial rows of the output
        (gm_conv2d_fwd_grouped_stats_bf16), for the stem BN's finalize."""
        lib = L.load()
        B, _, C0, H, W = x.shape
        K, _, R, S = weights[0].shape
        P, Q, Sp, Hp, Wp = _stem_geom(H, W, R, S, pad)
        dev = x.device
        xp = torch.empty(G * B, Hp, Wp // 2, 8, device=dev, dtype=BF)
        wp = torch.empty(G, K, R, Sp, 8, device=dev, dtype=BF)
        if G <= 4:
            stem_pack_grouped([x[:, g] for g in range(G)], weights, pad, xp, wp)  # one launch
        else:
            for g in range(G):
                stem_pack(x[:, g], weights[g], pad, xp=xp[g * B:(g + 1) * B], wp=wp[g])
        y = torch.empty(G * B, K, P, Q, device=dev, dtype=BF, memory_format=CL)
        d = _desc_hw(B, Hp, Wp // 2, 8, K, R, Sp, 2, 1, 0, 0)
        rows = lib.gm_conv_stem_stats_rows(ctypes.byref(d), G) if (stats is not None and FUSED_STEM_STATS) else 0
        if rows > 0:
            part = torch.empty(G, rows + 1, 128, device=dev, dtype=torch.float32)
            L.check(lib.gm_conv2d_fwd_grouped_stats_bf16(ctypes.byref(d), G, xp.data_ptr(), wp.data_ptr(),
                                                         K * R * Sp * 8, y.data_ptr(), part.data_ptr(), rows,
                                                         L.stream_of(dev)), "gm_conv2d_fwd_grouped_stats_bf16")
            stats["part"], stats["rows"] = part, rows
        else:
            L.check(lib.gm_conv2d_fwd_grouped_bf16(ctypes.byref(d), G, xp.data_ptr(), wp.data_ptr(), K * R * Sp * 8,
                                                   y.data_ptr(), 0, 0, L.stream_of(dev)), "gm_conv2d_fwd_grouped_bf16")
        ctx.save_for_backward(xp, *weights)
        ctx.meta = (G, B, R, S, Sp)
        # the stem BN + ReLU + max-pool backward hands its operands over (stats["bwd"]) instead of
        # writing dy when the weight gradient can form dy itself (gm_conv2d_wgrad_stem_bn_ok)
        ctx.link = stats
        if stats is not None:
            stats["stem_bn_ok"] = FUSED_STEM_WGRAD and lib.gm_conv2d_wgrad_stem_bn_ok(ctypes.byref(d), G) == 1
        return y

    @staticmethod
    def backward(ctx, gy):
        xp, *weights = ctx.saved_tensors
        G, B, R, S, Sp = ctx.meta
        want = [ctx.needs_input_grad[4 + g] for g in range(G)]
        if not any(want):
            return (None, None, None, None, *[None] * G)
        lib = L.load()
        bw = ctx.link.pop("bwd", None) if ctx.link is not None else None
        if bw is None:
            gy = _nhwc(gy.to(BF))
        dev = gy.device
        _, Hp, Wq, _ = xp.shape
        K, C0 = weights[0].shape[0], weights[0].shape[1]
        d = _desc_hw(B, Hp, Wq, 8, K, R, Sp, 2, 1, 0, 0)
        need = lib.gm_conv2d_wgrad_grouped_scratch(ctypes.byref(d), G)
        scratch = torch.empty(max(need, 16), device=dev, dtype=torch.uint8)
        dwp = torch.empty(G, K, R, Sp, 8, device=dev, dtype=torch.float32)
        if bw is not None:  # gy is a placeholder: dy is formed from the BN + pool operands
            src = L.StemBnSrc(bw["y"].data_ptr(), bw["dy_pool"].data_ptr(), bw["idx"].data_ptr(),
                              bw["fcoef"].data_ptr(), bw["fcoef"].stride(0), bw["bcoef"], bw["bcoef_gs"])
            L.check(lib.gm_conv2d_wgrad_stem_bn_grouped_bf16(ctypes.byref(d), G, ctypes.byref(src), xp.data_ptr(),
                                                             dwp.data_ptr(), K * R * Sp * 8, 0, scratch.data_ptr(),
                                                             need, L.stream_of(dev)),
                    "gm_conv2d_wgrad_stem_bn_grouped_bf16")
        else:
            L.check(lib.gm_conv2d_wgrad_grouped_bf16(ctypes.byref(d), G, gy.data_ptr(), xp.data_ptr(),
                                                     dwp.data_ptr(), K * R * Sp * 8, 8, 0, scratch.data_ptr(), need,
                                                     L.stream_of(dev)), "gm_conv2d_wgrad_grouped_bf16")
        tgts = [sink_target(w) if want[g] else None for g, w in enumerate(weights)]
        if all(t is not None and t[1] == tgts[0][1] and t[0].dtype == torch.float32
               and t[0].is_contiguous(memory_format=CL) for t in tgts):
            # every view's gradient sink at once: one crop launch into the [K][R][S][C0] memory
            ptrs = (ctypes.c_void_p * G)(*[t[0].data_ptr() for t in tgts])
            L.check(lib.gm_stem_dw_crop(dwp.data_ptr(), G, K, R, S, C0, Sp, ptrs, int(bool(tgts[0][1])),
                                        L.stream_of(dev)), "gm_stem_dw_crop")
            for w in weights:
                sink_done(w)
            return (None, None, None, None, *[None] * G)
        grads = []
        for g, w in enumerate(weights):
            if not want[g]:
                grads.append(None)
                continue
            dw = dwp[g].view(K, R, 2 * Sp, 4)[:, :, :S, :C0].permute(0, 3, 1, 2)  # [K,C0,R,S]
            tgt = tgts[g]  # (sink_target marks the gradient written: called once per step above)
            if tgt is not None:
                if tgt[1]:
                    tgt[0].add_(dw)
                else:
                    tgt[0].copy_(dw)
                sink_done(w)
                grads.append(None)
            else:
                grads.append(_like_param(dw, w))
        return (None, None, None, None, *grads)


class _VBNReluPoolFn(torch.autograd.Function):
    """pool(relu(BatchNorm_g(X_g))) per view group: one grouped statistics launch, one pool
    launch applying each group's coefficients (bn._BNReluPoolFn, stacked)."""

    @staticmethod
    def forward(ctx, X, G, bns, k, s, pad, stats, *params):
        lib = L.load()
        gammas, betas = params[:G], params[G:]
        xb = _nhwc(X.to(BF))
        GN, C, H, W = xb.shape
        N = GN // G
        M = N * H * W
        dev = xb.device
        sm = torch.empty(G, C, device=dev, dtype=torch.float32)
        si = torch.empty(G, C, device=dev, dtype=torch.float32)
        coef = torch.empty(G, 2 * C, device=dev, dtype=torch.float32)
        descs = [L.BnFwd(M, C, 1, xb[g * N:(g + 1) * N].data_ptr(), 0, 0, gammas[g].data_ptr(), betas[g].data_ptr(),
                         L.ptr(bn.running_mean), L.ptr(bn.running_var), float(bn.momentum), float(bn.eps),
                         sm[g].data_ptr(), si[g].data_ptr(), L.ptr(bn.num_batches_tracked), coef[g].data_ptr())
                 for g, bn in enumerate(bns)]
        st = L.stream_of(dev)
        if stats is not None and "part" in stats:  # partial rows from the stem convolution's epilogue
            L.check(lib.gm_bn_fwd_stats_finalize_grouped(L.arr(L.BnFwd, descs), G, stats["part"].data_ptr(),
                                                         stats["rows"], st), "gm_bn_fwd_stats_finalize_grouped")
        else:
            buf = _bn_scratch_g(dev, M, C, G)
            L.check(lib.gm_bn_fwd_stats_grouped_bf16(L.arr(L.BnFwd, descs), G, buf.data_ptr(), buf.numel(), st),
                    "gm_bn_fwd_stats_grouped_bf16")
        P, Q = (H + 2 * pad - k) // s + 1, (W + 2 * pad - k) // s + 1
        y = torch.empty(GN, C, P, Q, device=dev, dtype=BF, memory_format=CL)
        idx = torch.empty(GN, P, Q, C, device=dev, dtype=torch.uint8)
        # the selected raw x per pooled output: the fused backward's statistics pass reads it
        # (and the pooled gradient) instead of x, the gradient and the argmax
        fused_bwd = FUSED_STEM_BWD and (k, s, pad, C) == (3, 2, 1, 64)
        xsel = torch.empty(GN, P, Q, C, device=dev, dtype=BF) if fused_bwd else None
        ctx.xsel_on = STEM_XSEL
        d = L.PoolDesc(N, H, W, C, k, s, pad)
        L.check(lib.gm_bn_relu_maxpool2d_fwd_grouped_bf16(ctypes.byref(d), G, xb.data_ptr(), coef.data_ptr(),
                                                          y.data_ptr(), idx.data_ptr(), L.ptr(xsel), st),
                "gm_bn_relu_maxpool2d_fwd_grouped_bf16")
        ctx.save_for_backward(xb, coef, sm, si, idx, xsel, *gammas, *betas)
        ctx.meta = (G, k, s, pad)
        ctx.link = stats
        return y

    @staticmethod
    def backward(ctx, dy):
        flush_wgrads()  # the trunk's remaining weight gradients overlap the stem's backward
        lib = L.load()
        xb, coef, sm, si, idx, xsel, *prm = ctx.saved_tensors
        G, k, s, pad = ctx.meta
        gammas, betas = prm[:G], prm[G:]
        GN, C, H, W = xb.shape
        dy = _nhwc(dy.to(BF))
        want_w, want_b = any(ctx.needs_input_grad[7:7 + G]), any(ctx.needs_input_grad[7 + G:])
        if xsel is not None and (want_w or want_b):
            # the pool's input gradient is gathered inside the BN backward's two passes
            # (gm_bn_relu_maxpool2d_bwd_grouped_bf16): never written.  With the stem's fused weight
            # gradient (ctx.link["stem_bn_ok"]) only the statistics pass runs here and dx is never
            # written at all: the stem's backward forms it in its loader from the operands handed
            # over in ctx.link["bwd"]; the gradient returned for X is a placeholder it does not read
            N = GN // G
            M = N * H * W
            link = ctx.link if (ctx.needs_input_grad[0] and ctx.link is not None
                                and ctx.link.get("stem_bn_ok")) else None
            dx = None if link is not None else torch.empty_like(xb, memory_format=CL)
            dgs, dbs, acc, sunk = _bn_param_grads(gammas, betas, want_w, want_b)
            descs = [L.BnBwd(M, C, 1, 0, 0, xb[g * N:(g + 1) * N].data_ptr(), gammas[g].data_ptr(), sm[g].data_ptr(),
                             si[g].data_ptr(), dx[g * N:(g + 1) * N].data_ptr() if dx is not None else 0, 0,
                             dgs[g].data_ptr(), dbs[g].data_ptr(), int(acc), 0, coef[g].data_ptr())
                     for g in range(G)]
            buf = _bn_scratch_g(xb.device, M, C, G)
            d = L.PoolDesc(N, H, W, C, k, s, pad)
            if link is not None:
                bcoef, bgs = ctypes.c_void_p(), ctypes.c_longlong()
                L.check(lib.gm_bn_relu_maxpool2d_bwd_stats_grouped_bf16(
                    ctypes.byref(d), G, dy.data_ptr(), idx.data_ptr(), xsel.data_ptr() if ctx.xsel_on else 0,
                    L.arr(L.BnBwd, descs), buf.data_ptr(), buf.numel(), ctypes.byref(bcoef), ctypes.byref(bgs),
                    L.stream_of(xb.device)), "gm_bn_relu_maxpool2d_bwd_stats_grouped_bf16")
                link["bwd"] = dict(y=xb, dy_pool=dy, idx=idx, fcoef=coef, bcoef=bcoef.value, bcoef_gs=bgs.value,
                                   keep=buf)
                dx = torch.empty((), device=xb.device, dtype=xb.dtype).expand(xb.shape)
            else:
                L.check(lib.gm_bn_relu_maxpool2d_bwd_grouped_bf16(ctypes.byref(d), G, dy.data_ptr(), idx.data_ptr(),
                                                                  xsel.data_ptr() if ctx.xsel_on else 0,
                                                                  L.arr(L.BnBwd, descs), buf.data_ptr(),
                                                                  buf.numel(), L.stream_of(xb.device)),
                        "gm_bn_relu_maxpool2d_bwd_grouped_bf16")
            if sunk:
                for p in list(gammas) + list(betas):
                    sink_done(p)
                gw, gb = [None] * G, [None] * G
            else:
                gw = [t if want_w else None for t in dgs]
                gb = [t if want_b else None for t in dbs]
            return (dx if ctx.needs_input_grad[0] else None, None, None, None, None, None, None, *gw, *gb)
        dz = torch.empty_like(xb, memory_format=CL)
        d = L.PoolDesc(GN, H, W, C, k, s, pad)
        L.check(lib.gm_maxpool2d_bwd_bf16(ctypes.byref(d), dy.data_ptr(), idx.data_ptr(), dz.data_ptr(),
                                          L.stream_of(xb.device)), "gm_maxpool2d_bwd_bf16")
        dx, _, gw, gb = _bn_backward(dz, None, xb, G, gammas, betas, sm, si, True, False, coef, want_w, want_b)
        return (dx if ctx.needs_input_grad[0] else None, None, None, None, None, None, None, *gw, *gb)


def vstem(x, nets):
    """layer-1 input of every view, stacked: maxpool(relu(bn1(conv1(x[:, g])))) per net g."""
    G = len(nets)
    c0 = nets[0].conv1
    pool = nets[0].maxpool
    from .pool import _pair1
    k, s, p = (_pair1(getattr(pool, a)) for a in ("kernel_size", "stride", "padding"))
    stats = {}  # the stem convolution's BN partial rows, handed to the BN's finalize
    with torch.autocast("cuda", enabled=False):
        y = _VStemFn.apply(x, G, c0.padding[0], stats, *[n.conv1.weight for n in nets])
        bns = [n.bn1 for n in nets]
        return _VBNReluPoolFn.apply(y, G, bns, k, s, p, stats, *[b.weight for b in bns], *[b.bias for b in bns])


# ---- blocks and eligibility ---------------------------------------------------------

def vblock(blocks, X):
    """One ResNet block position of every view (BasicBlock.forward / Bottleneck.forward,
    resnet.py, stacked)."""
    b0 = blocks[0]
    join = GradJoin()
    ds = b0.downsample is not None
    join.masked_ok = not ds  # its consumers: conv1 (vconv takes a MaskedAddend) and the output BN

    def cbn(x, convs, bns, cjoin=None, link_in=None, link_out=None, res_link=None, **kw):
        # conv -> BatchNorm, the forward statistics from the conv's epilogue; link_out: this
        # BN (+ ReLU) feeds the next conv, whose input-gradient epilogue then sums this BN's
        # backward statistics (link_in of that conv); res_link: the downsample BN <-> the block
        # output BN whose residual it is (its only consumer)
        st = {"dgrad_link": link_in, "bn_link": link_out, "dz_link": res_link, "res_link": res_link}
        return vbn(vconv(x, convs, cjoin, stats=st), bns, stats=st, **kw)
    rl = {} if ds else None
    if ds:
        idt = cbn(X, [b.downsample[0] for b in blocks], [b.downsample[1] for b in blocks], join, res_link=rl)
    else:
        idt = X
    l1 = {}
    out = cbn(X, [b.conv1 for b in blocks], [b.bn1 for b in blocks], join, link_out=l1, relu=True)
    if hasattr(b0, "conv3"):  # Bottleneck
        l2 = {}
        out = cbn(out, [b.conv2 for b in blocks], [b.bn2 for b in blocks], link_in=l1, link_out=l2, relu=True)
        return cbn(out, [b.conv3 for b in blocks], [b.bn3 for b in blocks], link_in=l2, residual=idt, relu=True,
                   residual_join=None if ds else join, res_link=rl)
    return cbn(out, [b.conv2 for b in blocks], [b.bn2 for b in blocks], link_in=l1, residual=idt, relu=True,
               residual_join=None if ds else join, res_link=rl)


def vlayer(nets, i, X):
    """layer{i} of every view over the stacked X."""
    layers = [getattr(n, f"layer{i}") for n in nets]
    for j in range(len(layers[0])):
        X = vblock([lay[j] for lay in layers], X)
    return X


def usable(model, nets, x):
    """The stacked trunk applies: training-mode bf16 (input or autocast) on HIP, 2..16 views of
    one architecture with the pixel-pair stem, every BN tracking statistics with momentum."""
    from .bn import GMBatchNorm2d
    from .conv import GMConv2d
    if not (ENABLED and model.training and x.is_cuda and x.dim() == 5 and 2 <= len(nets) <= 16):
        return False
    if not (x.dtype == BF or (torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == BF)):
        return False
    if not torch.is_grad_enabled():
        return False
    sig = None
    for n in nets:
        if not n.training or not n.conv1.uses_pair_stem():
            return False
        mods = [m for m in n.modules() if isinstance(m, (GMConv2d, GMBatchNorm2d))]
        s = [(type(m).__name__, tuple(m.weight.shape)) for m in mods]
        if sig is None:
            sig = s
        elif s != sig:
            return False
        if any(isinstance(m, GMBatchNorm2d) and (m.momentum is None or not m.track_running_stats or not m.affine)
               for m in mods):
            return False
    return True
