"""BatchNorm2d (+ residual add + ReLU) of the ResNet trunk on the HIP kernels.

`GMBatchNorm2d` is an `nn.BatchNorm2d` (same parameters, buffers, names, init,
state_dict) whose forward takes two optional fusions used by the ResNet blocks:

    bn(x)                         == BatchNorm2d(x)
    bn(x, relu=True)              == relu(BatchNorm2d(x))
    bn(x, residual=r, relu=True)  == relu(BatchNorm2d(x) + r)

For CUDA inputs in training mode it runs `gm_bn_fwd_train_*` / `gm_bn_bwd_*`
(batch statistics, running-stat and num_batches_tracked updates inside the
kernel); in eval mode without autograd `gm_bn_fwd_infer_*`.  bf16 inputs (the
engine's trunk, autocast-bf16) take the bf16 kernels (single launch each way
where the grid can be co-resident); fp32 inputs - the reference's own
arithmetic - take the fp32 kernels, activations channels_last.  There is no
PyTorch batch_norm path: CPU tensors raise.  Reference: torchvision ResNet
BasicBlock/Bottleneck as used by src/model.py:53-56,65-106.
"""
import ctypes

import torch
import torch.nn as nn

from .streams import zeroed_scratch
from . import _lib as L
from .gradsink import sink_done, sink_target

CL = torch.channels_last

_scratch = {}

# ReLU BNs without a residual keep the forward's fp32 affine coefficients (2C floats)
# instead of y: the backward recomputes the mask x*sc + sh > 0 from x, which it reads
# anyway, so y is never read back (one bf16 activation read fewer in each of the two
# backward kernels).  (False keeps the y mask.)
MASK_FROM_X = True

# The stem's BN + ReLU + max-pool in one statistics launch and one pool launch
# (GMBatchNorm2d.relu_maxpool); False composes the two modules.
FUSE_POOL = True


def _get_scratch(device, M, C):
    """Per-(device, stream) BN scratch (ticket word + coefficients + partials),
    zeroed once at allocation; the kernels leave the ticket at zero.  One buffer
    per stream: the trunks run on separate streams concurrently (streams.py), and
    two BN launches in flight must not share tickets."""
    need = L.load().gm_bn_scratch(M, C)
    return zeroed_scratch(_scratch, device, need,
                          lambda old: max(need, 1 << 20) if old is None else max(need, 2 * old.numel()))


def _nhwc(t):
    return t if t.is_contiguous(memory_format=CL) else t.contiguous(memory_format=CL)


def _check_shape(x, C):
    if x.dim() != 4 or x.shape[1] != C:
        raise ValueError(f"expected [N,{C},H,W], got {tuple(x.shape)}")
    if C < 8 or C > 2048 or C & (C - 1):
        raise ValueError(f"HIP batchnorm needs C a power of two in [8, 2048], got {C}")


def _fn(lib, name, dtype):
    return getattr(lib, name + ("_f32" if dtype == torch.float32 else "_bf16"))


def bn_fwd_train(x, weight, bias, running_mean, running_var, nbt, momentum, eps, relu, residual, coef=None):
    """coef: optional fp32 [2C] tensor receiving the affine coefficients (sc, sh).
    x bf16 or fp32 (channels_last); the residual is cast to x's dtype."""
    lib = L.load()
    N, C, H, W = x.shape
    _check_shape(x, C)
    M = N * H * W
    x = _nhwc(x)
    if residual is not None:
        residual = _nhwc(residual.to(x.dtype))
    y = torch.empty_like(x, memory_format=CL)
    sm = torch.empty(C, device=x.device, dtype=torch.float32)
    si = torch.empty(C, device=x.device, dtype=torch.float32)
    buf = _get_scratch(x.device, M, C)
    p = L.BnFwd(M, C, int(relu), x.data_ptr(), L.ptr(residual), y.data_ptr(), weight.data_ptr(),
                bias.data_ptr(), L.ptr(running_mean), L.ptr(running_var), float(momentum), float(eps),
                sm.data_ptr(), si.data_ptr(), L.ptr(nbt), L.ptr(coef))
    L.check(_fn(lib, "gm_bn_fwd_train", x.dtype)(ctypes.byref(p), buf.data_ptr(), buf.numel(),
                                                 L.stream_of(x.device)), "gm_bn_fwd_train")
    return y, sm, si


def bn_fwd_infer(x, weight, bias, running_mean, running_var, eps, relu, residual):
    lib = L.load()
    N, C, H, W = x.shape
    _check_shape(x, C)
    M = N * H * W
    x = _nhwc(x)
    if residual is not None:
        residual = _nhwc(residual.to(x.dtype))
    y = torch.empty_like(x, memory_format=CL)
    buf = _get_scratch(x.device, M, C)
    p = L.BnFwd(M, C, int(relu), x.data_ptr(), L.ptr(residual), y.data_ptr(), weight.data_ptr(),
                bias.data_ptr(), running_mean.data_ptr(), running_var.data_ptr(), 0.0, float(eps), 0, 0, 0)
    L.check(_fn(lib, "gm_bn_fwd_infer", x.dtype)(ctypes.byref(p), buf.data_ptr(), buf.numel(),
                                                 L.stream_of(x.device)), "gm_bn_fwd_infer")
    return y


def bn_bwd(dy, y, x, weight, sm, si, relu, want_dres, dgamma, dbeta, accumulate, fwd_coef=None):
    """Returns (dx, dres); dgamma/dbeta are written (or added) in place.  With relu,
    the mask comes from y, or from x and the forward's coefficients when y is None."""
    lib = L.load()
    N, C, H, W = x.shape
    M = N * H * W
    dy = _nhwc(dy.to(x.dtype))
    dx = torch.empty_like(x, memory_format=CL)
    dres = torch.empty_like(x, memory_format=CL) if want_dres else None
    buf = _get_scratch(x.device, M, C)
    p = L.BnBwd(M, C, int(relu), dy.data_ptr(), L.ptr(y) if relu else 0, x.data_ptr(), weight.data_ptr(),
                sm.data_ptr(), si.data_ptr(), dx.data_ptr(), L.ptr(dres), dgamma.data_ptr(), dbeta.data_ptr(),
                int(accumulate), 0, L.ptr(fwd_coef))
    L.check(_fn(lib, "gm_bn_bwd", x.dtype)(ctypes.byref(p), buf.data_ptr(), buf.numel(), L.stream_of(x.device)),
            "gm_bn_bwd")
    return dx, dres


class _BNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, nbt, momentum, eps, relu, join=None,
                dtype=torch.bfloat16):
        ctx.join = join
        xb = _nhwc(x.to(dtype))
        maskx = relu and residual is None and MASK_FROM_X
        coef = torch.empty(2 * xb.shape[1], device=xb.device, dtype=torch.float32) if maskx else None
        y, sm, si = bn_fwd_train(xb, weight.detach(), bias.detach(), running_mean, running_var, nbt, momentum,
                                 eps, relu, residual, coef)
        ctx.save_for_backward(xb, y if relu and not maskx else coef, weight, bias, sm, si)
        ctx.maskx = maskx
        ctx.relu = relu
        ctx.has_res = residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        xb, y, weight, bias, sm, si = ctx.saved_tensors
        coef = None
        if ctx.maskx:
            y, coef = None, y
        want_dres = ctx.has_res and ctx.needs_input_grad[3]
        dx, gw, gb, dres = _bn_backward(dy, y, xb, weight, bias, sm, si, ctx.relu, want_dres, coef,
                                        ctx.needs_input_grad[1], ctx.needs_input_grad[2])
        dx = dx if ctx.needs_input_grad[0] else None
        if dres is not None and ctx.join is not None:  # the residual's gradient joins the block input's
            dres = ctx.join.contribute(lambda add: dres if add is None else dres + add)
        return dx, gw, gb, dres, None, None, None, None, None, None, None, None


def _bn_backward(dy, y, xb, weight, bias, sm, si, relu, want_dres, coef, want_w, want_b):
    """BN backward with the parameter gradients written straight into the gradient sink
    when the engine armed one (weight and bias share its state), else returned.
    Returns (dx, grad_weight, grad_bias, dres)."""
    C = xb.shape[1]
    tw = sink_target(weight) if want_w else None
    tb = sink_target(bias) if want_b else None
    if tw is not None and tb is not None and tw[1] == tb[1]:
        dgamma, dbeta, acc = tw[0], tb[0], tw[1]
        direct = True
    else:
        if tw is not None or tb is not None:  # mixed state: undo nothing, fall back to returned grads
            raise RuntimeError("GMBatchNorm2d: weight and bias must share one gradient sink state")
        dgamma = torch.empty(C, device=xb.device, dtype=torch.float32)
        dbeta = torch.empty(C, device=xb.device, dtype=torch.float32)
        acc, direct = False, False
    dx, dres = bn_bwd(dy, y, xb, weight.detach(), sm, si, relu, want_dres, dgamma, dbeta, acc, coef)
    if direct:
        sink_done(weight)
        sink_done(bias)
        return dx, None, None, dres
    return dx, (dgamma if want_w else None), (dbeta if want_b else None), dres


class _BNReluPoolFn(torch.autograd.Function):
    """relu(BatchNorm2d(x)) followed by MaxPool2d(k, s, pad) - the ResNet stem - with the
    normalised activation never materialised: one statistics launch
    (gm_bn_fwd_stats_bf16), then the pool applies the affine + ReLU on the fly
    (gm_bn_relu_maxpool2d_fwd_bf16); bit-identical to bn(x, relu=True) on the two-launch
    path followed by the max-pool.  Backward: the pool's gather (dz), then the BN
    backward with the ReLU mask recomputed from x and the forward's coefficients."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, nbt, momentum, eps, k, s, pad):
        lib = L.load()
        xb = _nhwc(x.to(torch.bfloat16))
        N, C, H, W = xb.shape
        _check_shape(xb, C)
        M = N * H * W
        sm = torch.empty(C, device=xb.device, dtype=torch.float32)
        si = torch.empty(C, device=xb.device, dtype=torch.float32)
        coef = torch.empty(2 * C, device=xb.device, dtype=torch.float32)
        buf = _get_scratch(xb.device, M, C)
        st = L.stream_of(xb.device)
        p = L.BnFwd(M, C, 1, xb.data_ptr(), 0, 0, weight.data_ptr(), bias.data_ptr(), L.ptr(running_mean),
                    L.ptr(running_var), float(momentum), float(eps), sm.data_ptr(), si.data_ptr(), L.ptr(nbt),
                    coef.data_ptr())
        L.check(lib.gm_bn_fwd_stats_bf16(ctypes.byref(p), buf.data_ptr(), buf.numel(), st), "gm_bn_fwd_stats_bf16")
        P, Q = (H + 2 * pad - k) // s + 1, (W + 2 * pad - k) // s + 1
        y = torch.empty(N, C, P, Q, device=xb.device, dtype=torch.bfloat16, memory_format=CL)
        idx = torch.empty(N, P, Q, C, device=xb.device, dtype=torch.uint8)
        d = L.PoolDesc(N, H, W, C, k, s, pad)
        L.check(lib.gm_bn_relu_maxpool2d_fwd_bf16(ctypes.byref(d), xb.data_ptr(), coef.data_ptr(), y.data_ptr(),
                                                  idx.data_ptr(), st), "gm_bn_relu_maxpool2d_fwd_bf16")
        ctx.save_for_backward(xb, coef, weight, bias, sm, si, idx)
        ctx.pool = (k, s, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = L.load()
        xb, coef, weight, bias, sm, si, idx = ctx.saved_tensors
        k, s, pad = ctx.pool
        N, C, H, W = xb.shape
        dy = _nhwc(dy.to(torch.bfloat16))
        dz = torch.empty_like(xb, memory_format=CL)
        d = L.PoolDesc(N, H, W, C, k, s, pad)
        L.check(lib.gm_maxpool2d_bwd_bf16(ctypes.byref(d), dy.data_ptr(), idx.data_ptr(), dz.data_ptr(),
                                          L.stream_of(xb.device)), "gm_maxpool2d_bwd_bf16")
        dx, gw, gb, _ = _bn_backward(dz, None, xb, weight, bias, sm, si, True, False, coef,
                                     ctx.needs_input_grad[1], ctx.needs_input_grad[2])
        dx = dx if ctx.needs_input_grad[0] else None
        return dx, gw, gb, None, None, None, None, None, None, None, None


def _use_bf16(x):
    return x.dtype == torch.bfloat16 or (
        torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16)


class GMBatchNorm2d(nn.BatchNorm2d):
    """nn.BatchNorm2d with optional fused residual add and ReLU (see module doc)."""

    def forward(self, x, residual=None, relu=False, residual_join=None):
        """residual_join: gradsink.GradJoin of the residual tensor (see conv.GMConv2d)."""
        C = self.num_features
        if not x.is_cuda:
            raise L.GreedyMMLError("GMBatchNorm2d: the trunk runs on libgreedymml_hip.so only (got a CPU tensor)")
        if not (self.affine and self.track_running_stats and x.dim() == 4 and 8 <= C <= 2048 and not (C & (C - 1))):
            raise L.GreedyMMLError("GMBatchNorm2d: needs affine, tracked running stats, [N,C,H,W] with C a power "
                                   f"of two in [8, 2048] (got C={C})")
        dt = torch.bfloat16 if _use_bf16(x) else torch.float32
        if self.training:
            if self.momentum is None:
                raise L.GreedyMMLError("GMBatchNorm2d: cumulative averaging (momentum=None) is not supported")
            join = None
            if (residual_join is not None and residual is not None and residual.requires_grad
                    and torch.is_grad_enabled()):
                residual_join.register()
                join = residual_join
            with torch.autocast("cuda", enabled=False):
                return _BNFn.apply(x, self.weight, self.bias, residual, self.running_mean, self.running_var,
                                   self.num_batches_tracked, self.momentum, self.eps, bool(relu), join, dt)
        if torch.is_grad_enabled() and (x.requires_grad or self.weight.requires_grad):
            raise L.GreedyMMLError("GMBatchNorm2d: eval-mode forward with autograd is not supported")
        return bn_fwd_infer(x.to(dt), self.weight, self.bias, self.running_mean, self.running_var,
                            self.eps, bool(relu), residual)

    def relu_maxpool(self, x, pool):
        """pool(relu(self(x))) - the ResNet stem.  Training on the bf16 trunk with the
        engine's max-pool takes the fused path (_BNReluPoolFn: the normalised activation
        is never written); anything else composes the two modules."""
        from .pool import GMMaxPool2d, _pair1
        C = self.num_features
        k, s, p = (_pair1(getattr(pool, a)) for a in ("kernel_size", "stride", "padding"))
        fused = (FUSE_POOL and self.training and x.is_cuda and _use_bf16(x) and isinstance(pool, GMMaxPool2d)
                 and None not in (k, s, p) and _pair1(pool.dilation) == 1 and not pool.ceil_mode
                 and not pool.return_indices and k <= 15 and 2 * p <= k and C % 8 == 0 and 8 <= C <= 2048
                 and not (C & (C - 1)) and self.affine and self.track_running_stats and self.momentum is not None
                 and x.dim() == 4 and x.shape[1] == C)
        if not fused:
            return pool(self(x, relu=True))
        with torch.autocast("cuda", enabled=False):
            return _BNReluPoolFn.apply(x, self.weight, self.bias, self.running_mean, self.running_var,
                                       self.num_batches_tracked, self.momentum, self.eps, k, s, p)
