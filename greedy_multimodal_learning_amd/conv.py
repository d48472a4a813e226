"""ResNet trunk convolutions on the bf16 MFMA implicit-GEMM kernels.

`GMConv2d` is an `nn.Conv2d` (same parameters, names, init and state_dict) whose
forward runs `gm_conv2d_fwd_bf16` and whose backward runs
`gm_conv2d_dgrad_bf16` + `gm_conv2d_wgrad_bf16` whenever it sees a bf16 input on
a HIP device (the engine's bf16 channels_last trunk, or autocast-bf16).  fp32
inputs (the fp32 parity mode) go through PyTorch's convolution (MIOpen).
Activations are channels_last (NHWC) bf16, weights are cast to bf16 KRSC per
step, weight gradients come back in fp32 in the parameter's layout.
"""
import ctypes

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib as L
from .gradsink import sink_done, sink_target

CL = torch.channels_last


def _desc(N, H, W, C, K, R, S, stride, pad):
    return L.ConvDesc(N, H, W, C, K, R, S, stride, pad)


def _nhwc(t):
    return t if t.is_contiguous(memory_format=CL) else t.contiguous(memory_format=CL)


def _pad_c(x, c):
    """[N,C,H,W] channels_last -> channels padded with zeros to c (e.g. RGB -> 8)."""
    N, C0, H, W = x.shape
    out = torch.empty(N, c, H, W, device=x.device, dtype=x.dtype, memory_format=CL).zero_()
    out[:, :C0].copy_(x)
    return out


def _cpad(c):
    p = 8
    while p < c:
        p *= 2
    return p


def conv_fwd(x, w, stride, pad):
    """x [N,C,H,W] bf16 channels_last, w [K,C,R,S] bf16 channels_last -> y [N,K,P,Q]."""
    lib = L.load()
    N, C, H, W = x.shape
    K, _, R, S = w.shape
    P = (H + 2 * pad - R) // stride + 1
    Q = (W + 2 * pad - S) // stride + 1
    y = torch.empty(N, K, P, Q, device=x.device, dtype=torch.bfloat16, memory_format=CL)
    d = _desc(N, H, W, C, K, R, S, stride, pad)
    L.check(lib.gm_conv2d_fwd_bf16(ctypes.byref(d), x.data_ptr(), w.data_ptr(), y.data_ptr(),
                                   L.stream_of(x.device)), "gm_conv2d_fwd_bf16")
    return y


def conv_dgrad(dy, w, H, W, stride, pad):
    lib = L.load()
    N, K, P, Q = dy.shape
    _, C, R, S = w.shape
    wt = torch.empty(C, K, R, S, device=w.device, dtype=torch.bfloat16, memory_format=CL)
    L.check(lib.gm_conv_weight_transpose_bf16(w.data_ptr(), wt.data_ptr(), K, R * S, C,
                                              L.stream_of(w.device)), "gm_conv_weight_transpose_bf16")
    dx = torch.empty(N, C, H, W, device=dy.device, dtype=torch.bfloat16, memory_format=CL)
    d = _desc(N, H, W, C, K, R, S, stride, pad)
    L.check(lib.gm_conv2d_dgrad_bf16(ctypes.byref(d), dy.data_ptr(), wt.data_ptr(), dx.data_ptr(),
                                     L.stream_of(dy.device)), "gm_conv2d_dgrad_bf16")
    return dx


def conv_wgrad(dy, x, R, S, stride, pad, c_real, out=None, accumulate=False):
    """fp32 weight gradient [K,c_real,R,S] (channels_last); written into `out`
    (a KRSC-contiguous gradient buffer, added to if accumulate) when given."""
    lib = L.load()
    N, C, H, W = x.shape
    K = dy.shape[1]
    d = _desc(N, H, W, C, K, R, S, stride, pad)
    need = lib.gm_conv2d_wgrad_scratch(ctypes.byref(d))
    scratch = torch.empty(max(need, 16), device=x.device, dtype=torch.uint8)
    if out is None:
        dw = torch.empty(K, c_real, R, S, device=x.device, dtype=torch.float32, memory_format=CL)
    else:
        if (tuple(out.shape) != (K, c_real, R, S) or out.dtype != torch.float32
                or not out.is_contiguous(memory_format=CL)):
            raise ValueError("conv_wgrad: out must be fp32 [K,C,R,S] channels_last")
        dw = out
    L.check(lib.gm_conv2d_wgrad_bf16(ctypes.byref(d), dy.data_ptr(), x.data_ptr(), dw.data_ptr(), c_real,
                                     int(accumulate), scratch.data_ptr(), need, L.stream_of(x.device)),
            "gm_conv2d_wgrad_bf16")
    return dw


def weight_prep(weight, Cp, transposed):
    """fp32 [K,C,R,S] parameter -> bf16 KRSC copy padded to Cp channels (+ optional
    channel-transposed copy [Cp,K,R,S] for dgrad), one kernel."""
    lib = L.load()
    K, C, R, S = weight.shape
    w32 = weight.detach()
    if w32.dtype != torch.float32:
        w32 = w32.float()
    w32 = _nhwc(w32)
    wb = torch.empty(K, Cp, R, S, device=w32.device, dtype=torch.bfloat16, memory_format=CL)
    wt = torch.empty(Cp, K, R, S, device=w32.device, dtype=torch.bfloat16, memory_format=CL) if transposed else None
    L.check(lib.gm_conv_weight_prep_bf16(w32.data_ptr(), K, R * S, C, Cp, wb.data_ptr(), L.ptr(wt),
                                         L.stream_of(w32.device)), "gm_conv_weight_prep_bf16")
    return wb, wt


_prepped = {}  # weight data_ptr -> (wb, wt): bf16 copies made by an active WeightPrep


class WeightPrep:
    """bf16 copies of every GMConv2d weight of a model, made by ONE launch per step
    (gm_conv_weight_prep_multi_bf16) instead of one prep launch per convolution.
    The engine runs it at the start of a step and activates the copies for that
    step's forward only (a weight changed outside the step is never served stale)."""

    def __init__(self, model):
        lib = L.load()
        convs = [m for m in model.modules() if isinstance(m, GMConv2d)]
        dev = next(model.parameters()).device
        specs, total = [], 0
        for m in convs:
            K, C, R, S = m.weight.shape
            Cp = _cpad(C)
            want_t = C >= 8  # the stem's input (RGB) never needs an input gradient
            n = K * R * S * Cp
            specs.append((m.weight, K, C, R, S, Cp, want_t, total))
            total += n * (2 if want_t else 1)
        self.buf = torch.empty(max(total, 1), device=dev, dtype=torch.bfloat16)
        self.copies = []
        items, tiles = [], 0
        for (w, K, C, R, S, Cp, want_t, off) in specs:
            n = K * R * S * Cp
            wb = self.buf[off:off + n].view(K, R, S, Cp).permute(0, 3, 1, 2)
            wt = self.buf[off + n:off + 2 * n].view(Cp, R, S, K).permute(0, 3, 1, 2) if want_t else None
            self.copies.append((w, wb, wt))
            items.append(L.WPrep(0, wb.data_ptr(), L.ptr(wt), K, R * S, C, Cp, tiles, 0))
            tiles += lib.gm_wprep_tiles(K, R * S, Cp)
        self.items = items
        self.tiles = tiles
        self.table = None
        self._ptrs = None

    def _refresh_table(self):
        """(Re)build the device table when parameter storage moved (FlatParams)."""
        ptrs = tuple(w.data_ptr() for (w, _, _) in self.copies)
        if self.table is not None and ptrs == self._ptrs:
            return
        for it, (w, _, _), p in zip(self.items, self.copies, ptrs):
            if w.dtype != torch.float32 or not w.is_contiguous(memory_format=CL):
                raise RuntimeError("WeightPrep: conv weights must be fp32 channels_last (KRSC)")
            it.w = p
        raw = bytes(L.arr(L.WPrep, self.items))
        host = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
        self.table = host.to(self.buf.device)
        self._ptrs = ptrs

    def run(self):
        if not self.copies:
            return
        self._refresh_table()
        L.check(L.load().gm_conv_weight_prep_multi_bf16(self.table.data_ptr(), len(self.items), self.tiles,
                                                        L.stream_of(self.buf.device)),
                "gm_conv_weight_prep_multi_bf16")

    def activate(self):
        for (w, wb, wt) in self.copies:
            _prepped[w.data_ptr()] = (wb, wt)

    @staticmethod
    def deactivate():
        _prepped.clear()


def conv_dgrad_t(dy, wt, H, W, stride, pad):
    """dgrad from an already transposed bf16 weight wt [C,K,R,S] (channels_last)."""
    lib = L.load()
    N, K, P, Q = dy.shape
    C, _, R, S = wt.shape
    dx = torch.empty(N, C, H, W, device=dy.device, dtype=torch.bfloat16, memory_format=CL)
    d = _desc(N, H, W, C, K, R, S, stride, pad)
    L.check(lib.gm_conv2d_dgrad_bf16(ctypes.byref(d), dy.data_ptr(), wt.data_ptr(), dx.data_ptr(),
                                     L.stream_of(dy.device)), "gm_conv2d_dgrad_bf16")
    return dx


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride, pad):
        C0 = x.shape[1]
        Cp = _cpad(C0)
        xb = _nhwc(x.to(torch.bfloat16))
        if Cp != C0:
            xb = _pad_c(xb, Cp)
        need_dx = ctx.needs_input_grad[0]
        pre = _prepped.get(weight.data_ptr()) if _prepped else None
        if pre is not None and (pre[1] is not None or not need_dx):
            wb, wt = pre
        else:
            wb, wt = weight_prep(weight, Cp, need_dx)
        y = conv_fwd(xb, wb, stride, pad)
        ctx.save_for_backward(xb, wt, weight)
        ctx.meta = (stride, pad, C0, x.shape[2], x.shape[3], weight.shape[2], weight.shape[3])
        return y

    @staticmethod
    def backward(ctx, gy):
        xb, wt, weight = ctx.saved_tensors
        stride, pad, C0, H, W, R, S = ctx.meta
        gy = _nhwc(gy.to(torch.bfloat16))
        dx = None
        if ctx.needs_input_grad[0]:
            dx = conv_dgrad_t(gy, wt, H, W, stride, pad)
            if dx.shape[1] != C0:
                dx = dx[:, :C0]
        dw = None
        if ctx.needs_input_grad[1]:
            tgt = sink_target(weight)
            if tgt is not None and tgt[0].is_contiguous(memory_format=CL):
                conv_wgrad(gy, xb, R, S, stride, pad, C0, out=tgt[0], accumulate=tgt[1])
                sink_done(weight)
            else:
                if tgt is not None:
                    raise RuntimeError("GMConv2d: in-place gradient buffer must be channels_last")
                dw = conv_wgrad(gy, xb, R, S, stride, pad, C0)
        return dx, dw, None, None


def _use_hip(x):
    if not x.is_cuda:
        return False
    if x.dtype == torch.bfloat16:
        return True
    return torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16


class GMConv2d(nn.Conv2d):
    """nn.Conv2d whose bf16 path runs on libgreedymml_hip.so (groups=1, no bias,
    square stride/padding, dilation 1 - the ResNet trunk's convolutions)."""

    def forward(self, x):
        if (_use_hip(x) and self.groups == 1 and self.bias is None and self.dilation == (1, 1)
                and self.stride[0] == self.stride[1] and self.padding[0] == self.padding[1]
                and self.padding_mode == "zeros"):
            with torch.autocast("cuda", enabled=False):
                return _ConvFn.apply(x, self.weight, self.stride[0], self.padding[0])
        return F.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation, self.groups)
