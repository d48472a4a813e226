"""ResNet trunk convolutions on the hand-written MFMA implicit-GEMM kernels.

`GMConv2d` is an `nn.Conv2d` (same parameters, names, init and state_dict) whose
forward and backward run on libgreedymml_hip.so for every HIP input:

  * bf16 (the engine's channels_last trunk, or autocast-bf16): `gm_conv2d_fwd_bf16`
    + `gm_conv2d_dgrad_bf16` + `gm_conv2d_wgrad_bf16` (v_mfma_f32_32x32x16_bf16);
    activations channels_last bf16, weights cast to bf16 KRSC per step;
  * fp32 (the reference's own arithmetic: src/framework.py:146-148 feeds fp32
    tensors with no autocast): `gm_conv2d_f32` fwd / dgrad / wgrad on the exact-f32
    MFMA (v_mfma_f32_32x32x2_f32), activations channels_last fp32, any channel
    count (the RGB stem unpadded).

Weight gradients come back in fp32 in the parameter's layout (or are written in
place through the gradient sink).  There is no vendor-library path: a CPU tensor
or an unsupported configuration raises.
"""
import ctypes

import torch
import torch.nn as nn

from .streams import zeroed_scratch
from . import _lib as L
from .gradsink import sink_done, sink_target

CL = torch.channels_last


def _desc(N, H, W, C, K, R, S, stride, pad):
    return L.ConvDesc(N, H, W, C, K, R, S, stride, pad)


def _nhwc(t):
    return t if t.is_contiguous(memory_format=CL) else t.contiguous(memory_format=CL)


def _like_param(g, p):
    """A weight gradient in the parameter's own strides (what AccumulateGrad and the
    gate's flat norm pass expect), copying only when the element order differs."""
    if g.stride() == p.stride():
        return g
    out = torch.empty_strided(p.shape, p.stride(), device=g.device, dtype=g.dtype)
    out.copy_(g)
    return out


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


_splitk_ws = {}


def _splitk(device, d, dgrad):
    """Split-K workspace of this (device, stream): (pointer, bytes), zeroed once at
    allocation (the kernels leave their turnstile words at zero); per stream because
    the two view trunks run concurrently (streams.py)."""
    need = L.load().gm_conv2d_splitk_ws_bytes(ctypes.byref(d), int(dgrad))
    if need == 0:
        return 0, 0
    buf = zeroed_scratch(_splitk_ws, device, need, lambda old: (need + (1 << 20) - 1) >> 20 << 20)
    return buf.data_ptr(), buf.numel()


@L.on_fault_reset
def _reset_splitk_ws():
    """A timed-out turnstile can leave a flag word mid-sequence: zero every workspace."""
    for buf in _splitk_ws.values():
        buf.zero_()
    torch.cuda.synchronize()


def conv_fwd(x, w, stride, pad):
    """x [N,C,H,W] bf16 channels_last, w [K,C,R,S] bf16 channels_last -> y [N,K,P,Q]."""
    lib = L.load()
    N, C, H, W = x.shape
    K, _, R, S = w.shape
    P = (H + 2 * pad - R) // stride + 1
    Q = (W + 2 * pad - S) // stride + 1
    y = torch.empty(N, K, P, Q, device=x.device, dtype=torch.bfloat16, memory_format=CL)
    d = _desc(N, H, W, C, K, R, S, stride, pad)
    ws, nb = _splitk(x.device, d, False)
    L.check(lib.gm_conv2d_fwd_ex_bf16(ctypes.byref(d), x.data_ptr(), w.data_ptr(), y.data_ptr(), ws, nb,
                                      L.stream_of(x.device)), "gm_conv2d_fwd_ex_bf16")
    return y


def conv_dgrad(dy, w, H, W, stride, pad):
    lib = L.load()
    N, K, P, Q = dy.shape
    _, C, R, S = w.shape
    wt = torch.empty(C, K, R, S, device=w.device, dtype=torch.bfloat16, memory_format=CL)
    L.check(lib.gm_conv_weight_transpose_bf16(w.data_ptr(), wt.data_ptr(), K, R * S, C,
                                              L.stream_of(w.device)), "gm_conv_weight_transpose_bf16")
    return conv_dgrad_t(dy, wt, H, W, stride, pad)


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


def _desc_hw(N, H, W, C, K, R, S, sh, sw, ph, pw):
    return L.ConvDescHW(N, H, W, C, K, R, S, sh, sw, ph, pw)


# ---- ResNet stem on a pixel-pair view -------------------------------------------
# A 7x7/s2 convolution of an RGB image wastes most of an MFMA K-slice if every tap is
# one 8-channel (3 real) chunk: K = 49 x 8 = 392 for 147 real products.  With the
# input as zero-bordered 4-channel pixels, two horizontally adjacent pixels form ONE
# 16-byte (8-channel) element, and the stride-2 filter becomes a 7 x 4 filter over
# pairs with strides (2, 1) and no padding: K = 7 x 4 x 8 = 224, every tap in range
# (the border is real zeros), half the input bytes.  The weights are re-packed to
# [K][R][S/2][2 x 4] per step (a 25 KB tensor).

def stem_pair_ok(C0, R, S, stride, pad):
    return C0 <= 4 and stride == 2 and R <= 8 and S <= 8 and pad < R and pad < S


def _stem_geom(H, W, R, S, pad):
    P = (H + 2 * pad - R) // 2 + 1
    Q = (W + 2 * pad - S) // 2 + 1
    Sp = (S + 1) // 2
    Hp = max(2 * (P - 1) + R, pad + H)
    Wp = max(2 * (Q - 1) + 2 * Sp, pad + W)
    Wp += Wp & 1
    return P, Q, Sp, Hp, Wp


def stem_pack_input(x, R, S, pad):
    """x [N,C0<=4,H,W] -> zero-bordered pair view [N,8,Hp,Wp/2] (channels_last bf16)."""
    N, C0, H, W = x.shape
    P, Q, Sp, Hp, Wp = _stem_geom(H, W, R, S, pad)
    xp = torch.zeros(N, Hp, Wp, 4, device=x.device, dtype=torch.bfloat16)
    xp[:, pad:pad + H, pad:pad + W, :C0] = x.permute(0, 2, 3, 1)
    return xp.view(N, Hp, Wp // 2, 8).permute(0, 3, 1, 2)


def stem_pack_weight(weight):
    """fp32 [K,C0,R,S] -> bf16 pair-packed [K,8,R,Sp] (channels_last: [K][R][Sp][2x4])."""
    K, C0, R, S = weight.shape
    Sp = (S + 1) // 2
    wp = torch.zeros(K, R, 2 * Sp, 4, device=weight.device, dtype=torch.bfloat16)
    wp[:, :, :S, :C0] = weight.detach().permute(0, 2, 3, 1)
    return wp.view(K, R, Sp, 8).permute(0, 3, 1, 2)


def stem_pack(x, weight, pad, xp=None, wp=None):
    """(stem_pack_input(x), stem_pack_weight(weight)) in one launch (gm_stem_pack_bf16);
    xp [N,Hp,Wp/2,8] / wp [K,R,Sp,8] bf16 dense outputs may be given (a view group's
    slice of the stacked trunk's buffers)."""
    N, C0, H, W = x.shape
    K, _, R, S = weight.shape
    P, Q, Sp, Hp, Wp = _stem_geom(H, W, R, S, pad)
    if x.dtype not in (torch.float32, torch.bfloat16):
        x = x.float()
    w = weight.detach()
    if w.dtype != torch.float32:
        w = w.float()
    if xp is None:
        xp = torch.empty(N, Hp, Wp // 2, 8, device=x.device, dtype=torch.bfloat16)
    if wp is None:
        wp = torch.empty(K, R, Sp, 8, device=x.device, dtype=torch.bfloat16)
    if (tuple(xp.shape) != (N, Hp, Wp // 2, 8) or tuple(wp.shape) != (K, R, Sp, 8) or not xp.is_contiguous()
            or not wp.is_contiguous()):
        raise ValueError("stem_pack: output buffers must be dense [N,Hp,Wp/2,8] / [K,R,Sp,8]")
    p = L.StemPack(x.data_ptr(), L.GM_BF16 if x.dtype == torch.bfloat16 else L.GM_F32, N, C0, H, W, pad,
                   *x.stride(), Hp, Wp, xp.data_ptr(), w.data_ptr(), K, R, S, wp.data_ptr(), *w.stride())
    L.check(L.load().gm_stem_pack_bf16(ctypes.byref(p), L.stream_of(x.device)), "gm_stem_pack_bf16")
    return xp.permute(0, 3, 1, 2), wp.permute(0, 3, 1, 2)


def stem_pack_grouped(xs, weights, pad, xp, wp):
    """stem_pack for G views in ONE launch (gm_stem_pack_grouped_bf16): view g's input xs[g]
    [N,C0,H,W] (any strides, fp32 or bf16, every view the same) and fp32 weight weights[g] into
    xp[g*N:(g+1)*N] ([G*N,Hp,Wp/2,8] dense bf16) and wp[g] ([G,K,R,Sp,8])."""
    G = len(xs)
    N, C0, H, W = xs[0].shape
    K, _, R, S = weights[0].shape
    P, Q, Sp, Hp, Wp = _stem_geom(H, W, R, S, pad)
    if tuple(xp.shape) != (G * N, Hp, Wp // 2, 8) or tuple(wp.shape) != (G, K, R, Sp, 8) or \
            not xp.is_contiguous() or not wp.is_contiguous():
        raise ValueError("stem_pack_grouped: outputs must be dense [G*N,Hp,Wp/2,8] / [G,K,R,Sp,8]")
    descs, keep = [], []
    for g, (x, w) in enumerate(zip(xs, weights)):
        if x.dtype not in (torch.float32, torch.bfloat16):
            x = x.float()
        w = w.detach()
        if w.dtype != torch.float32:
            w = w.float()
        keep += [x, w]
        descs.append(L.StemPack(x.data_ptr(), L.GM_BF16 if x.dtype == torch.bfloat16 else L.GM_F32, N, C0, H, W,
                                pad, *x.stride(), Hp, Wp, xp[g * N:(g + 1) * N].data_ptr(), w.data_ptr(), K, R, S,
                                wp[g].data_ptr(), *w.stride()))
    L.check(L.load().gm_stem_pack_grouped_bf16(L.arr(L.StemPack, descs), G, L.stream_of(xs[0].device)),
            "gm_stem_pack_grouped_bf16")


def stem_fwd(xp, wp, P, Q):
    lib = L.load()
    N, _, Hp, Wq = xp.shape
    K, _, R, Sp = wp.shape
    if (Hp - R) // 2 + 1 != P or Wq - Sp + 1 != Q:
        raise ValueError(f"stem pair view {tuple(xp.shape)} does not give a {P}x{Q} output")
    y = torch.empty(N, K, P, Q, device=xp.device, dtype=torch.bfloat16, memory_format=CL)
    d = _desc_hw(N, Hp, Wq, 8, K, R, Sp, 2, 1, 0, 0)
    L.check(lib.gm_conv2d_fwd_hw_bf16(ctypes.byref(d), xp.data_ptr(), wp.data_ptr(), y.data_ptr(),
                                      L.stream_of(xp.device)), "gm_conv2d_fwd_hw_bf16")
    return y


class _StemFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, pad):
        K, C0, R, S = weight.shape
        N, _, H, W = x.shape
        P, Q, Sp, Hp, Wp = _stem_geom(H, W, R, S, pad)
        xp, wp = stem_pack(x, weight, pad)
        y = stem_fwd(xp, wp, P, Q)
        ctx.save_for_backward(xp, weight)
        ctx.meta = (R, S, Sp)
        return y

    @staticmethod
    def backward(ctx, gy):
        xp, weight = ctx.saved_tensors
        R, S, Sp = ctx.meta
        if not ctx.needs_input_grad[1]:
            return None, None, None
        lib = L.load()
        gy = _nhwc(gy.to(torch.bfloat16))
        N, _, Hp, Wq = xp.shape
        K, C0 = weight.shape[0], weight.shape[1]
        d = _desc_hw(N, Hp, Wq, 8, K, R, Sp, 2, 1, 0, 0)
        need = lib.gm_conv2d_wgrad_hw_scratch(ctypes.byref(d))
        scratch = torch.empty(max(need, 16), device=xp.device, dtype=torch.uint8)
        dwp = torch.empty(K, R, Sp, 8, device=xp.device, dtype=torch.float32)
        L.check(lib.gm_conv2d_wgrad_hw_bf16(ctypes.byref(d), gy.data_ptr(), xp.data_ptr(), dwp.data_ptr(), 8, 0,
                                            scratch.data_ptr(), need, L.stream_of(xp.device)),
                "gm_conv2d_wgrad_hw_bf16")
        dw = dwp.view(K, R, 2 * Sp, 4)[:, :, :S, :C0].permute(0, 3, 1, 2)  # [K,C0,R,S] view of KRSC
        tgt = sink_target(weight)
        if tgt is not None:
            if tgt[1]:
                tgt[0].add_(dw)
            else:
                tgt[0].copy_(dw)
            sink_done(weight)
            return None, None, None
        return None, _like_param(dw, weight), None


_prepped = {}  # weight data_ptr -> (wb, wt): bf16 copies made by an active WeightPrep


class WeightPrep:
    """bf16 copies of every GMConv2d weight of a model, made by ONE launch per step
    (gm_conv_weight_prep_multi_bf16) instead of one prep launch per convolution.
    The engine runs it at the start of a step and activates the copies for that
    step's forward only (a weight changed outside the step is never served stale)."""

    def __init__(self, model):
        lib = L.load()
        convs = [m for m in model.modules() if isinstance(m, GMConv2d) and not m.uses_pair_stem()]
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


def conv_dgrad_t(dy, wt, H, W, stride, pad, addend=None, inplace=False):
    """dgrad from an already transposed bf16 weight wt [C,K,R,S] (channels_last);
    addend (bf16 [N,C,H,W] channels_last): dx = dgrad + addend in the epilogue, written
    over the addend itself when inplace (a strided dgrad then needs no pass that copies
    the addend to the pixels its parity classes do not cover)."""
    lib = L.load()
    N, K, P, Q = dy.shape
    C, _, R, S = wt.shape
    d = _desc(N, H, W, C, K, R, S, stride, pad)
    ws, nb = _splitk(dy.device, d, True)
    if addend is not None:
        if (tuple(addend.shape) != (N, C, H, W) or addend.dtype != torch.bfloat16
                or not addend.is_contiguous(memory_format=CL)):
            raise ValueError("conv dgrad addend must be a bf16 channels_last tensor shaped like dx")
    if inplace and addend is not None:
        dx = addend
    else:
        dx = torch.empty(N, C, H, W, device=dy.device, dtype=torch.bfloat16, memory_format=CL)
    L.check(lib.gm_conv2d_dgrad_add_bf16(ctypes.byref(d), dy.data_ptr(), wt.data_ptr(), dx.data_ptr(),
                                         L.ptr(addend), ws, nb, L.stream_of(dy.device)), "gm_conv2d_dgrad_add_bf16")
    return dx


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride, pad, join=None):
        ctx.join = join
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
            if ctx.join is not None and wt.shape[0] == C0:
                # the pending addend is this join's own tensor: summed in place
                dx = ctx.join.contribute(lambda add: conv_dgrad_t(gy, wt, H, W, stride, pad, addend=add, inplace=True))
            else:
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
                dw = _like_param(dw, weight)
        return dx, dw, None, None, None


def _use_hip(x):
    if not x.is_cuda:
        return False
    if x.dtype == torch.bfloat16:
        return True
    return torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16


# ---- reference-precision (fp32) path ------------------------------------------------

def conv_f32(mode, d, x=None, w=None, dy=None, out=None, addend=None, accumulate=False):
    """One gm_conv2d_f32 call (mode L.GM_CONV_FWD / _DGRAD / _WGRAD) on channels_last
    fp32 tensors; `out` must be preallocated in its NHWC / KRSC layout."""
    lib = L.load()
    p = L.ConvF32(mode, d, L.ptr(x), L.ptr(w), L.ptr(dy), L.ptr(out), L.ptr(addend), int(accumulate), 0)
    need = lib.gm_conv2d_f32_scratch(ctypes.byref(p))
    dev = out.device
    scratch = torch.empty(max(need, 16), device=dev, dtype=torch.uint8) if need else None
    L.check(lib.gm_conv2d_f32(ctypes.byref(p), L.ptr(scratch), need, L.stream_of(dev)), "gm_conv2d_f32")
    return out


def _f32_cl(t):
    t = t if t.dtype == torch.float32 else t.float()
    return _nhwc(t)


class _ConvF32Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride, pad, join=None):
        ctx.join = join
        xc = _f32_cl(x)
        wk = _f32_cl(weight.detach())  # KRSC (a no-op for the engine's channels_last parameters)
        N, C, H, W = xc.shape
        K, _, R, S = wk.shape
        P, Q = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1
        y = torch.empty(N, K, P, Q, device=xc.device, dtype=torch.float32, memory_format=CL)
        conv_f32(L.GM_CONV_FWD, _desc(N, H, W, C, K, R, S, stride, pad), x=xc, w=wk, out=y)
        ctx.save_for_backward(xc, wk, weight)
        ctx.meta = (stride, pad)
        return y

    @staticmethod
    def backward(ctx, gy):
        xc, wk, weight = ctx.saved_tensors
        stride, pad = ctx.meta
        gy = _f32_cl(gy)
        N, C, H, W = xc.shape
        K, _, R, S = wk.shape
        d = _desc(N, H, W, C, K, R, S, stride, pad)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            def dgrad(add):
                out = torch.empty(N, C, H, W, device=gy.device, dtype=torch.float32, memory_format=CL)
                if add is not None:
                    add = _f32_cl(add)
                return conv_f32(L.GM_CONV_DGRAD, d, w=wk, dy=gy, out=out, addend=add)
            dx = ctx.join.contribute(dgrad) if ctx.join is not None else dgrad(None)
        if ctx.needs_input_grad[1]:
            tgt = sink_target(weight)
            if tgt is not None:
                if not (tgt[0].is_contiguous(memory_format=CL) and tgt[0].dtype == torch.float32):
                    raise RuntimeError("GMConv2d: in-place gradient buffer must be fp32 channels_last")
                conv_f32(L.GM_CONV_WGRAD, d, x=xc, dy=gy, out=tgt[0], accumulate=tgt[1])
                sink_done(weight)
            else:
                dw = torch.empty(K, C, R, S, device=gy.device, dtype=torch.float32, memory_format=CL)
                conv_f32(L.GM_CONV_WGRAD, d, x=xc, dy=gy, out=dw)
                dw = _like_param(dw, weight)
        return dx, dw, None, None, None


class GMConv2d(nn.Conv2d):
    """nn.Conv2d whose bf16 path runs on libgreedymml_hip.so (groups=1, no bias,
    square stride/padding, dilation 1 - the ResNet trunk's convolutions)."""

    pair_stem = True

    def _hip_ok(self):
        return (self.groups == 1 and self.bias is None and self.dilation == (1, 1)
                and self.stride[0] == self.stride[1] and self.padding[0] == self.padding[1]
                and self.padding_mode == "zeros")

    def uses_pair_stem(self):
        """The RGB stem (<= 4 input channels, stride 2) runs on the pixel-pair view."""
        K, C0, R, S = self.weight.shape
        return self.pair_stem and self._hip_ok() and stem_pair_ok(C0, R, S, self.stride[0], self.padding[0])

    def forward(self, x, grad_join=None):
        """grad_join: a gradsink.GradJoin shared with the other consumers of x (the
        ResNet block input), so x's gradient is summed inside the dgrad epilogue."""
        if not x.is_cuda:
            raise L.GreedyMMLError("GMConv2d: the trunk runs on libgreedymml_hip.so only (got a CPU tensor)")
        if not self._hip_ok():
            raise L.GreedyMMLError("GMConv2d: only groups=1, no bias, square stride/padding, dilation 1, "
                                   "zero padding (the ResNet trunk's convolutions)")
        bf16 = _use_hip(x)
        with torch.autocast("cuda", enabled=False):
            if grad_join is not None and x.requires_grad and torch.is_grad_enabled():
                grad_join.register()
            else:
                grad_join = None
            if not bf16:
                return _ConvF32Fn.apply(x, self.weight, self.stride[0], self.padding[0], grad_join)
            if self.uses_pair_stem() and not x.requires_grad:
                if grad_join is not None:  # never: the stem input needs no gradient
                    raise RuntimeError("GMConv2d: pair stem with a gradient join")
                return _StemFn.apply(x, self.weight, self.padding[0])
            return _ConvFn.apply(x, self.weight, self.stride[0], self.padding[0], grad_join)
