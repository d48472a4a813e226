"""Classification heads of all branches and the branch-summed loss on the HIP kernels.

`pooled_linear(fs, fcs)` == `[fc(flatten(avgpool(f), 1)) for f, fc in zip(fs, fcs)]`
(the ResNet head, reference src/model.py:53-56 / torchvision resnet `avgpool` + `fc`)
for every branch at once:

    forward : gm_mmtm_spatial_reduce (global average pool of all branches, one launch,
              fp32) + gm_gemm_f32 (the fc layers, one launch)          -> fp32 logits
    backward: gm_gemm_f32 (dW, db, d_pooled of all branches, one launch; dW/db written
              in place through the gradient sink) + gm_mmtm_channel_scale (d_pooled/HW
              broadcast over the map, one launch)

`branch_xent(logits, y)` == train.py:22-29 `blend_loss` (sum over the branches of the
batch-mean cross-entropy): gm_xent_fwd / gm_xent_bwd, one launch each.

Both replace ~40 small PyTorch launches (pool reductions, dtype casts, hipBLASLt
GEMMs, log_softmax / nll_loss forward and backward, fills, adds) at the step's end.
The logits are fp32 (the reference's are fp32; autocast would give bf16).
"""
import torch

from . import _lib as L
from . import ops
from .gradsink import sink_done, sink_target

CL = torch.channels_last



_ZERO = {}


def zero_row(dev, C):
    """A persistent [1, C] fp32 zero row (the head backward's zero scale operand): made once,
    ideally before any graph capture (BalancedStep does), so no fill launch per step."""
    key = (str(dev), C)
    z = _ZERO.get(key)
    if z is None:
        z = torch.zeros(1, C, device=dev, dtype=torch.float32)
        _ZERO[key] = z
    return z

def head_ok(fs, fcs):
    """The fused head applies to bf16 or fp32 channels_last CUDA maps of one shape with fp32 fc."""
    f0 = fs[0]
    if not (f0.is_cuda and f0.dim() == 4 and f0.dtype in (torch.bfloat16, torch.float32)):
        return False
    for f, fc in zip(fs, fcs):
        if (f.shape != f0.shape or f.dtype != f0.dtype or not f.is_contiguous(memory_format=CL)
                or fc.bias is None or fc.weight.dtype != torch.float32 or not fc.weight.is_cuda
                or fc.weight.shape[1] != f0.shape[1]):
            return False
    return f0.shape[2] * f0.shape[3] > 1 or f0.is_contiguous()


def _grad_buf(prm, shape, want):
    """(tensor to write, accumulate, sunk) for a parameter gradient."""
    if not want:
        return None, False, False
    tgt = sink_target(prm)
    if tgt is not None:
        t, acc = tgt
        if not t.is_contiguous() or tuple(t.shape) != tuple(shape):
            raise RuntimeError(f"head: in-place gradient buffer must be a contiguous {tuple(shape)}")
        return t, acc, True
    return torch.empty(*shape, device=prm.device, dtype=torch.float32), False, False


class _PooledLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, nb, stacked, *args):
        """stacked: args end with ONE [nb*B, C, H, W] tensor (the view-batched trunk's,
        branch i = rows i*B..), whose gradient then comes back as one tensor."""
        ws, bs, fs = args[:nb], args[nb:2 * nb], args[2 * nb:]
        ctx.stacked = stacked
        if stacked:
            X = fs[0]
            Bs = X.shape[0] // nb
            fs = [X[i * Bs:(i + 1) * Bs] for i in range(nb)]
        B, C, H, W = fs[0].shape
        HW = H * W
        N = ws[0].shape[0]
        dev = fs[0].device
        lay = L.GM_NHWC if HW > 1 else L.GM_NCHW
        dt = L.GM_F32 if fs[0].dtype == torch.float32 else L.GM_BF16
        pooled = torch.empty(nb, B, C, device=dev, dtype=torch.float32)
        ops.spatial_reduce([dict(x=f, C=C, HW=HW, out=pooled[i], ld_out=C, scale=1.0 / HW) for i, f in enumerate(fs)],
                           B, dt, lay, dev)
        logits = torch.empty(nb, B, N, device=dev, dtype=torch.float32)
        ops.gemm([dict(M=B, N=N, segs=[(C, ops.Op(pooled[i], C, 1), ops.Op(ws[i].detach(), 1, C))], C=logits[i],
                       ld_c=N, bias=bs[i].detach()) for i in range(nb)], dev)
        ctx.nb, ctx.shape, ctx.lay, ctx.dt = nb, (B, C, H, W), lay, dt
        ctx.params = list(ws) + list(bs)
        ctx.save_for_backward(pooled, *ws, *(args[2 * nb:] if stacked else fs))
        return tuple(logits[i] for i in range(nb))

    @staticmethod
    def backward(ctx, *dls):
        nb = ctx.nb
        pooled, rest = ctx.saved_tensors[0], ctx.saved_tensors[1:]
        ws, fs = rest[:nb], rest[nb:]
        B, C, H, W = ctx.shape
        gX = None
        if ctx.stacked:
            X = fs[0]
            fs = [X[i * B:(i + 1) * B] for i in range(nb)]
        HW = H * W
        N = ws[0].shape[0]
        dev = pooled.device
        live = [i for i in range(nb) if dls[i] is not None]
        dl = {i: dls[i].float().contiguous() for i in live}
        need = ctx.needs_input_grad
        probs, sunk = [], []
        gw, gb, dp = [None] * nb, [None] * nb, {}
        for i in live:
            w_t, w_acc, w_s = _grad_buf(ctx.params[i], (N, C), need[2 + i])
            b_t, b_acc, b_s = _grad_buf(ctx.params[nb + i], (N,), need[2 + nb + i])
            if w_t is not None:  # dW[n,c] = sum_b dl[b,n] pooled[b,c]
                probs.append(dict(M=N, N=C, segs=[(B, ops.Op(dl[i], 1, N), ops.Op(pooled[i], C, 1))], C=w_t,
                                  ld_c=C, accumulate=int(w_acc)))
                if w_s:
                    sunk.append(ctx.params[i])
                else:
                    gw[i] = w_t
            if b_t is not None:  # db[n] = sum_b dl[b,n]
                probs.append(dict(M=1, N=N, segs=[(B, ops.ONES, ops.Op(dl[i], N, 1))], C=b_t, ld_c=N,
                                  accumulate=int(b_acc)))
                if b_s:
                    sunk.append(ctx.params[nb + i])
                else:
                    gb[i] = b_t
            if need[2 + 2 * nb + (0 if ctx.stacked else i)]:  # d_pooled[b,c] = sum_n dl[b,n] W[n,c]
                dp[i] = torch.empty(B, C, device=dev, dtype=torch.float32)
                probs.append(dict(M=B, N=C, segs=[(N, ops.Op(dl[i], N, 1), ops.Op(ws[i].detach(), C, 1))],
                                  C=dp[i], ld_c=C))
        if probs:
            ops.gemm(probs, dev)
        gf = [None] * nb
        if ctx.stacked and dp:
            gX = torch.empty_like(ctx.saved_tensors[-1],
                                  memory_format=CL if ctx.lay == L.GM_NHWC else torch.contiguous_format)
            for i in range(nb):
                if i not in dp:  # a branch without a logits gradient: its rows get zeros
                    gX[i * B:(i + 1) * B].zero_()
        if dp:
            zero = zero_row(dev, C)
            sc = []
            for i, d in dp.items():
                gf[i] = gX[i * B:(i + 1) * B] if gX is not None else torch.empty_like(
                    fs[i], memory_format=CL if ctx.lay == L.GM_NHWC else torch.contiguous_format)
                # df = 0 * f + d_pooled / HW (the mean's gradient broadcast over the map)
                sc.append(dict(x=fs[i], y=gf[i], C=C, HW=HW, s=zero, ld_s=0, a=d, ld_a=C, alpha=1.0 / HW))
            ops.channel_scale(sc, B, ctx.dt, ctx.lay, dev)
        for prm in sunk:
            sink_done(prm)
        if ctx.stacked:
            return (None, None, *gw, *gb, gX)
        return (None, None, *gw, *gb, *gf)


def pooled_linear(fs, fcs):
    """Logits (fp32 [B, N]) of every branch: fc_i(flatten(avgpool(f_i)))."""
    nb = len(fs)
    with torch.autocast("cuda", enabled=False):
        return list(_PooledLinearFn.apply(nb, False, *[fc.weight for fc in fcs], *[fc.bias for fc in fcs], *fs))


def pooled_linear_stacked(X, fcs):
    """pooled_linear over the view-batched trunk's stacked map X ([nb*B, C, H, W]): same
    logits, one stacked input gradient."""
    nb = len(fcs)
    with torch.autocast("cuda", enabled=False):
        return list(_PooledLinearFn.apply(nb, True, *[fc.weight for fc in fcs], *[fc.bias for fc in fcs], X))


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, *logits):
        nb = len(logits)
        B, N = logits[0].shape
        x = _joined(logits)
        if x is None:
            x = torch.stack(logits).contiguous()
        lse = torch.empty(nb * B, device=x.device, dtype=torch.float32)
        loss = torch.empty((), device=x.device, dtype=torch.float32)
        L.check(L.load().gm_xent_fwd(x.data_ptr(), nb, B, N, y.data_ptr(), lse.data_ptr(), loss.data_ptr(),
                                     L.stream_of(x.device)), "gm_xent_fwd")
        ctx.save_for_backward(x, lse, y)
        return loss

    @staticmethod
    def backward(ctx, g):
        x, lse, y = ctx.saved_tensors
        nb, B, N = x.shape
        g = g.float().contiguous()
        dx = torch.empty_like(x)
        L.check(L.load().gm_xent_bwd(x.data_ptr(), lse.data_ptr(), nb, B, N, y.data_ptr(), g.data_ptr(),
                                     dx.data_ptr(), L.stream_of(x.device)), "gm_xent_bwd")
        return (None, *[dx[i] for i in range(nb)])


def _joined(logits):
    """[nb, B, N] tensor the logits are consecutive rows of (pooled_linear's output), or None."""
    base = logits[0]._base
    if base is None or base.dim() != 3 or base.shape[0] != len(logits) or not base.is_contiguous():
        return None
    for i, o in enumerate(logits):
        if o._base is not base or o.data_ptr() != base[i].data_ptr() or not o.is_contiguous():
            return None
    return base


def xent_ok(logits, y):
    x0 = logits[0]
    return (x0.is_cuda and x0.dim() == 2 and y.is_cuda and y.dtype == torch.int64 and y.dim() == 1
            and y.shape[0] == x0.shape[0]
            and all(o.dtype == torch.float32 and o.shape == x0.shape for o in logits))


def branch_xent(logits, y):
    """sum_i cross_entropy(logits[i], y) (batch mean) in one launch each way."""
    with torch.autocast("cuda", enabled=False):
        return _XentFn.apply(y.contiguous(), *logits)
