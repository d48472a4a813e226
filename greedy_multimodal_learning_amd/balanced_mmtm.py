"""MMTM squeeze-excite fusion on MI355X: drop-in for the reference's
`src.balanced_mmtm` module API.

`MMTM_mitigate(dim_visual, dim_skeleton, ratio, device=0, SEonly=False,
shareweight=False)` keeps the reference's constructor, parameter names
(fc_squeeze / fc_squeeze_{visual,skeleton} / fc_visual / fc_skeleton /
fc_excite), public attributes (`running_avg_weight_visual`,
`running_avg_weight_skeleton`, `step`) and
`forward(visual, skeleton, return_scale, return_squeezed_mps,
turnoff_cross_modal_flow, average_squeezemaps, curation_mode, caring_modality)
-> (Y_v, Y_s, scales|None, squeeze_array|None)` (reference
src/balanced_mmtm.py:15-154), including its quirks:

* both running averages track the VISUAL scale's batch mean (`:113-116`);
* every forward (also eval / no_grad) advances them and `step` (`:118`);
* curation replaces the caring modality's scale by its running average, so that
  branch's excite FC receives no gradient (`:135-152`);
* `return_squeezed_mps` outside the normal mode raises UnboundLocalError (`:123-124`).

The arithmetic runs in libgreedymml_hip.so: spatial squeeze and its backward
(LDS/wave reductions), the joint FC chain on fp32 MFMA, the running-average
update and the channel re-scale.  Activations may be fp32 or bf16, NCHW or
channels_last; the FC chain is always fp32.
"""
import torch
import torch.nn as nn

from . import _lib as L
from . import ops
from .gradsink import sink_done, sink_target
from .ops import ONES, Op

# position of each parameter among _MMTMFunction.forward's inputs (ctx.needs_input_grad)
_GRAD_INDEX = {"w_sq": 2, "b_sq": 3, "w_sq_v": 4, "b_sq_v": 5, "w_sq_s": 6, "b_sq_s": 7,
               "w_v": 8, "b_v": 9, "w_s": 10, "b_s": 11}

NORMAL, TURNOFF, SEONLY = 0, 1, 2


def _as_f32(t, dev):
    return t.detach().to(device=dev, dtype=torch.float32).contiguous()


def _state_f32(t, dev):
    """Running-average state as a dense fp32 tensor on `dev` (updated in place)."""
    if t.device != dev or t.dtype != torch.float32 or not t.is_contiguous():
        t = t.to(device=dev, dtype=torch.float32).contiguous()
    return t


def _step_counter(mod, dev):
    """Device copy of the module's `step` (int32 [1]); re-seeded from the host value
    whenever the host attribute was changed from outside."""
    sd = getattr(mod, "_step_dev", None)
    if sd is None or sd.device != dev or getattr(mod, "_step_mirror", None) != mod.step:
        sd = torch.full((1,), int(mod.step), dtype=torch.int32, device=dev)
        mod._step_dev = sd
        mod._step_mirror = mod.step
    return sd


class _MMTMFunction(torch.autograd.Function):
    """Y_v, Y_s = MMTM(X_v, X_s; fc weights).  Extra outputs e_v, e_s, sq are
    non-differentiable side results (scales / squeezed maps for recording)."""

    @staticmethod
    def forward(ctx, xv, xs, w_sq, b_sq, w_sq_v, b_sq_v, w_sq_s, b_sq_s, w_v, b_v, w_s, b_s, cfg):
        ctx.grad_off = 0
        return _mmtm_forward(ctx, xv, xs, w_sq, b_sq, w_sq_v, b_sq_v, w_sq_s, b_sq_s, w_v, b_v, w_s, b_s, cfg)

    @staticmethod
    def backward(ctx, gyv, gys, _ge_v, _ge_s, _gsq):
        return _mmtm_backward(ctx, gyv, gys)


class _MMTMStackedFn(torch.autograd.Function):
    """The same site over the view-batched trunk's stacked activation X = [X_v; X_s]
    (vtrunk.py: [2B, C, H, W], view 0 first): Y = [Y_v; Y_s] is written as one stacked
    tensor and the backward returns one stacked dX - no split / concatenation copies
    between the grouped trunk launches and the site."""

    @staticmethod
    def forward(ctx, X, w_sq, b_sq, w_sq_v, b_sq_v, w_sq_s, b_sq_s, w_v, b_v, w_s, b_s, cfg):
        ctx.grad_off = -1
        B = X.shape[0] // 2
        Y = torch.empty_like(X)
        _, _, e_v, e_s, sq = _mmtm_forward(ctx, X[:B], X[B:], w_sq, b_sq, w_sq_v, b_sq_v, w_sq_s, b_sq_s, w_v, b_v,
                                           w_s, b_s, cfg, outs=(Y[:B], Y[B:]))
        return Y, e_v, e_s, sq

    @staticmethod
    def backward(ctx, gY, _ge_v, _ge_s, _gsq):
        xv = ctx.saved_tensors[0]
        B = xv.shape[0]
        fmt = torch.channels_last if xv.dim() == 4 and xv.is_contiguous(memory_format=torch.channels_last) \
            else torch.contiguous_format
        dX = torch.empty((2 * B,) + tuple(xv.shape[1:]), device=xv.device, dtype=xv.dtype, memory_format=fmt)
        gyv, gys = (None, None) if gY is None else (gY[:B], gY[B:])
        res = _mmtm_backward(ctx, gyv, gys, outs=(dX[:B], dX[B:]))
        return (dX,) + res[2:]


def _mmtm_forward(ctx, xv, xs, w_sq, b_sq, w_sq_v, b_sq_v, w_sq_s, b_sq_s, w_v, b_v, w_s, b_s, cfg, outs=None):
    dev = xv.device
    B, Cv, Cs = xv.shape[0], xv.shape[1], xs.shape[1]
    HWv, HWs = xv[0, 0].numel(), xs[0, 0].numel()
    lay = cfg["layout"]
    dt = ops._DT[xv.dtype]
    mode, share = cfg["mode"], cfg["share"]
    f32 = dict(device=dev, dtype=torch.float32)
    C2 = Cv + Cs
    # ---- squeeze: sq = [GAP(X_v) | GAP(X_s)]  [B, Cv+Cs] fp32
    sq = torch.empty(B, C2, **f32)
    ops.spatial_reduce([dict(x=xv, C=Cv, HW=HWv, out=sq, ld_out=C2, scale=1.0 / HWv),
                        dict(x=xs, C=Cs, HW=HWs, out=sq, out_off=Cv, ld_out=C2,
                             scale=1.0 / HWs)], B, dt, lay, dev)
    # ---- joint FC: z (relu)
    if mode == NORMAL:
        Cz = w_sq.shape[0]
        z_v = torch.empty(B, Cz, **f32)
        z_s = z_v
        ops.gemm([dict(M=B, N=Cz, segs=[(C2, Op(sq, C2, 1), Op(w_sq, 1, C2))], C=z_v, ld_c=Cz,
                       bias=b_sq, act=1)], dev)
    elif mode == TURNOFF:
        Cz = w_sq.shape[0]
        avg_v, avg_s = cfg["avg_v"], cfg["avg_s"]
        z_v, z_s = torch.empty(B, Cz, **f32), torch.empty(B, Cz, **f32)
        ops.gemm([
            dict(M=B, N=Cz, segs=[(Cv, Op(sq, C2, 1), Op(w_sq, 1, C2)),
                                  (Cs, Op(avg_s, 0, 1), Op(w_sq, 1, C2, off=Cv))],
                 C=z_v, ld_c=Cz, bias=b_sq, act=1),
            dict(M=B, N=Cz, segs=[(Cv, Op(avg_v, 0, 1), Op(w_sq, 1, C2)),
                                  (Cs, Op(sq, C2, 1, off=Cv), Op(w_sq, 1, C2, off=Cv))],
                 C=z_s, ld_c=Cz, bias=b_sq, act=1)], dev)
    else:
        Cz = w_sq_v.shape[0]
        z_v, z_s = torch.empty(B, Cz, **f32), torch.empty(B, Cz, **f32)
        ops.gemm([
            dict(M=B, N=Cz, segs=[(Cv, Op(sq, C2, 1), Op(w_sq_v, 1, Cv))], C=z_v, ld_c=Cz,
                 bias=b_sq_v, act=1),
            dict(M=B, N=Cz, segs=[(Cs, Op(sq, C2, 1, off=Cv), Op(w_sq_s, 1, Cs))], C=z_s,
                 ld_c=Cz, bias=b_sq_s, act=1)], dev)
    # ---- excite: e_m = sigmoid(W_m z_m + b_m)
    wv_, bv_ = (w_v, b_v)
    ws_, bs_ = (w_v, b_v) if share else (w_s, b_s)
    e_v, e_s = torch.empty(B, Cv, **f32), torch.empty(B, Cs, **f32)
    ops.gemm([dict(M=B, N=Cv, segs=[(Cz, Op(z_v, Cz, 1), Op(wv_, 1, Cz))], C=e_v, ld_c=Cv,
                   bias=bv_, act=2),
              dict(M=B, N=Cs, segs=[(Cz, Op(z_s, Cz, 1), Op(ws_, 1, Cz))], C=e_s, ld_c=Cs,
                   bias=bs_, act=2)], dev)
    # ---- running averages (both from e_v: reference quirk) + step, in place with
    # the step counter in device memory (graph-capturable)
    ra_v, ra_s = cfg["ra_v"], cfg["ra_s"]
    ops.running_avg_dev(e_v, ra_v, ra_s, cfg["step_dev"])
    # ---- effective scales (curation substitutes the running average)
    cur, caring = cfg["curation"], cfg["caring"]
    sv, ld_sv, live_v = e_v, Cv, True
    ss, ld_ss, live_s = e_s, Cs, True
    gate = cfg.get("gate")
    if gate is None:
        if cur and caring == 0:
            sv, ld_sv, live_v = ra_v, 0, False
        elif cur and caring == 1:
            ss, ld_ss, live_s = ra_s, 0, False
    # on-device gate (engine): the flags live in device memory, so one captured step serves
    # every curation setting; the channel scale reads the substituted modality's running
    # average in place of its scale rows, and backward zeroes that modality's excitation
    # gradient inside the squeeze-backward launch (gm_mmtm_*_gated)
    yv, ys = (torch.empty_like(xv), torch.empty_like(xs)) if outs is None else outs
    ops.channel_scale([dict(x=xv, y=yv, C=Cv, HW=HWv, s=sv, ld_s=ld_sv),
                       dict(x=xs, y=ys, C=Cs, HW=HWs, s=ss, ld_s=ld_ss)], B, dt, lay, dev,
                      gate=gate, alt=(ra_v, ra_s))
    ctx.save_for_backward(xv, xs, sq, z_v, z_s, e_v, e_s, sv, ss,
                          w_sq, w_sq_v, w_sq_s, wv_, ws_)
    # the parameters themselves (leaves), for in-place gradient delivery (gradsink)
    ctx.params = {"w_sq": w_sq, "b_sq": b_sq, "w_sq_v": w_sq_v, "b_sq_v": b_sq_v, "w_sq_s": w_sq_s,
                  "b_sq_s": b_sq_s, "w_v": w_v, "b_v": b_v, "w_s": w_s, "b_s": b_s}
    ctx.meta = (B, Cv, Cs, Cz, HWv, HWs, lay, dt, mode, share, live_v, live_s,
                ld_sv, ld_ss, cfg.get("avg_v"), cfg.get("avg_s"), cfg["zero_curated"], gate, ra_v, ra_s)
    ctx.mark_non_differentiable(e_v, e_s, sq)
    ctx.set_materialize_grads(False)  # no zero-filled grads for the side outputs
    return yv, ys, e_v, e_s, sq


def _mmtm_backward(ctx, gyv, gys, outs=None):
    (xv, xs, sq, z_v, z_s, e_v, e_s, sv, ss, w_sq, w_sq_v, w_sq_s, wv_, ws_) = ctx.saved_tensors
    (B, Cv, Cs, Cz, HWv, HWs, lay, dt, mode, share, live_v, live_s,
     ld_sv, ld_ss, avg_v, avg_s, zero_curated, gate, ra_v, ra_s) = ctx.meta
    dev = xv.device
    f32 = dict(device=dev, dtype=torch.float32)
    C2 = Cv + Cs
    # parameter gradients: written by the GEMMs straight into the engine's flat
    # gradient buffer when the parameter is sink-managed (no AccumulateGrad add)
    sunk, acc_of = {}, {}

    def gbuf(key, *shape):
        prm = ctx.params.get(key)
        tgt = (sink_target(prm) if prm is not None and ctx.needs_input_grad[_GRAD_INDEX[key] + ctx.grad_off]
               else None)
        if tgt is not None:
            t, acc = tgt
            if t.is_contiguous() and tuple(t.shape) == shape:
                sunk[key] = prm
                acc_of[id(t)] = acc
                return t
            raise RuntimeError(f"MMTM {key}: in-place gradient buffer must be a contiguous {shape}")
        return torch.empty(*shape, **f32)

    def gemm_acc(problems):
        for q in problems:
            if acc_of.get(id(q["C"])):
                q["accumulate"] = 1
        ops.gemm(problems, dev)
    if gyv is None:
        gyv = torch.zeros_like(xv)
    if gys is None:
        gys = torch.zeros_like(xs)
    gyv = ops.as_layout(gyv.to(xv.dtype), lay)
    gys = ops.as_layout(gys.to(xs.dtype), lay)
    # ---- da_m = (sum_hw dY_m X_m) * e_m (1 - e_m) for live modalities
    da_v = torch.empty(B, Cv, **f32) if live_v else None
    da_s = torch.empty(B, Cs, **f32) if live_s else None
    probs = []
    if live_v:
        probs.append(dict(x=xv, dy=gyv, C=Cv, HW=HWv, out=da_v, ld_out=Cv, e=e_v, ld_e=Cv))
    if live_s:
        probs.append(dict(x=xs, dy=gys, C=Cs, HW=HWs, out=da_s, ld_out=Cs, e=e_s, ld_e=Cs))
    if probs:  # on-device gate: the substituted modality's da is zeroed in the same launch
        ops.spatial_reduce(probs, B, dt, lay, dev, gate=gate)
    # ---- excite FC grads + dz
    g = {}
    probs = []
    if share:
        if live_v or live_s:
            g["w_v"] = gbuf("w_v", Cv, Cz)
            g["b_v"] = gbuf("b_v", Cv)
            segw = [(B, Op(da, 1, Cv), Op(z, Cz, 1)) for da, z in ((da_v, z_v), (da_s, z_s))
                    if da is not None]
            segb = [(B, ONES, Op(da, Cv, 1)) for da in (da_v, da_s) if da is not None]
            probs += [dict(M=Cv, N=Cz, segs=segw, C=g["w_v"], ld_c=Cz),
                      dict(M=1, N=Cv, segs=segb, C=g["b_v"], ld_c=Cv)]
    else:
        for key, da, z, C in (("v", da_v, z_v, Cv), ("s", da_s, z_s, Cs)):
            if da is None:
                continue
            g["w_" + key] = gbuf("w_" + key, C, Cz)
            g["b_" + key] = gbuf("b_" + key, C)
            probs += [dict(M=C, N=Cz, segs=[(B, Op(da, 1, C), Op(z, Cz, 1))], C=g["w_" + key],
                           ld_c=Cz),
                      dict(M=1, N=C, segs=[(B, ONES, Op(da, C, 1))], C=g["b_" + key], ld_c=C)]
    dz_v = dz_s = None
    if mode == NORMAL:
        segs = [(C, Op(da, C, 1), Op(w, Cz, 1)) for da, w, C in ((da_v, wv_, Cv), (da_s, ws_, Cs))
                if da is not None]
        if segs:
            dz_v = torch.empty(B, Cz, **f32)
            dz_s = dz_v
            probs.append(dict(M=B, N=Cz, segs=segs, C=dz_v, ld_c=Cz, mask=z_v, ld_mask=Cz))
    else:
        if da_v is not None:
            dz_v = torch.empty(B, Cz, **f32)
            probs.append(dict(M=B, N=Cz, segs=[(Cv, Op(da_v, Cv, 1), Op(wv_, Cz, 1))], C=dz_v,
                              ld_c=Cz, mask=z_v, ld_mask=Cz))
        if da_s is not None:
            dz_s = torch.empty(B, Cz, **f32)
            probs.append(dict(M=B, N=Cz, segs=[(Cs, Op(da_s, Cs, 1), Op(ws_, Cz, 1))], C=dz_s,
                              ld_c=Cz, mask=z_s, ld_mask=Cz))
    if probs:
        gemm_acc(probs)
    # ---- squeeze FC grads + dsq
    probs = []
    dsq = None
    if mode == NORMAL and dz_v is not None:
        dsq = torch.empty(B, C2, **f32)
        g["w_sq"] = gbuf("w_sq", Cz, C2)
        g["b_sq"] = gbuf("b_sq", Cz)
        probs += [dict(M=Cz, N=C2, segs=[(B, Op(dz_v, 1, Cz), Op(sq, C2, 1))], C=g["w_sq"], ld_c=C2),
                  dict(M=1, N=Cz, segs=[(B, ONES, Op(dz_v, Cz, 1))], C=g["b_sq"], ld_c=Cz),
                  dict(M=B, N=C2, segs=[(Cz, Op(dz_v, Cz, 1), Op(w_sq, C2, 1))], C=dsq, ld_c=C2)]
    elif mode == TURNOFF and (dz_v is not None or dz_s is not None):
        dsq = torch.zeros(B, C2, **f32) if (dz_v is None or dz_s is None) else torch.empty(B, C2, **f32)
        g["w_sq"] = gbuf("w_sq", Cz, C2)
        g["b_sq"] = gbuf("b_sq", Cz)
        # fc_squeeze saw in_v = [sq_v | avg_s] and in_s = [avg_v | sq_s]
        left = [(B, Op(dz, 1, Cz), src) for dz, src in
                ((dz_v, Op(sq, C2, 1)), (dz_s, Op(avg_v, 0, 1))) if dz is not None]
        right = [(B, Op(dz, 1, Cz), src) for dz, src in
                 ((dz_v, Op(avg_s, 0, 1)), (dz_s, Op(sq, C2, 1, off=Cv))) if dz is not None]
        probs += [dict(M=Cz, N=Cv, segs=left, C=g["w_sq"], ld_c=C2),
                  dict(M=Cz, N=Cs, segs=right, C=g["w_sq"], c_off=Cv, ld_c=C2),
                  dict(M=1, N=Cz, segs=[(B, ONES, Op(dz, Cz, 1)) for dz in (dz_v, dz_s)
                                        if dz is not None], C=g["b_sq"], ld_c=Cz)]
        if dz_v is not None:
            probs.append(dict(M=B, N=Cv, segs=[(Cz, Op(dz_v, Cz, 1), Op(w_sq, C2, 1))], C=dsq,
                              ld_c=C2))
        if dz_s is not None:
            probs.append(dict(M=B, N=Cs, segs=[(Cz, Op(dz_s, Cz, 1), Op(w_sq, C2, 1, off=Cv))],
                              C=dsq, c_off=Cv, ld_c=C2))
    elif mode == SEONLY and (dz_v is not None or dz_s is not None):
        dsq = torch.zeros(B, C2, **f32) if (dz_v is None or dz_s is None) else torch.empty(B, C2, **f32)
        for key, dz, w, C, off in (("v", dz_v, w_sq_v, Cv, 0), ("s", dz_s, w_sq_s, Cs, Cv)):
            if dz is None:
                continue
            g["w_sq_" + key] = gbuf("w_sq_" + key, Cz, C)
            g["b_sq_" + key] = gbuf("b_sq_" + key, Cz)
            probs += [dict(M=Cz, N=C, segs=[(B, Op(dz, 1, Cz), Op(sq, C2, 1, off=off))],
                           C=g["w_sq_" + key], ld_c=C),
                      dict(M=1, N=Cz, segs=[(B, ONES, Op(dz, Cz, 1))], C=g["b_sq_" + key], ld_c=Cz),
                      dict(M=B, N=C, segs=[(Cz, Op(dz, Cz, 1), Op(w, C, 1))], C=dsq, c_off=off,
                           ld_c=C2)]
    if probs:
        gemm_acc(probs)
    # ---- dX_m = dY_m * s_m + dsq_m / HW
    dxv, dxs = (torch.empty_like(xv), torch.empty_like(xs)) if outs is None else outs
    pv = dict(x=gyv, y=dxv, C=Cv, HW=HWv, s=sv, ld_s=ld_sv)
    ps = dict(x=gys, y=dxs, C=Cs, HW=HWs, s=ss, ld_s=ld_ss)
    if dsq is not None:
        pv.update(a=dsq, ld_a=C2, alpha=1.0 / HWv)
        ps.update(a=dsq, a_off=Cv, ld_a=C2, alpha=1.0 / HWs)
    ops.channel_scale([pv, ps], B, dt, lay, dev, gate=gate, alt=(ra_v, ra_s))

    for prm in sunk.values():  # delivered in place: fire the engine's per-parameter hook
        sink_done(prm)

    def out(key, shape_like):
        if key in sunk:
            return None
        t = g.get(key)
        if t is None and zero_curated and shape_like is not None:
            return torch.zeros_like(shape_like)
        return t
    return (dxv, dxs,
            out("w_sq", w_sq), out("b_sq", None if w_sq is None else w_sq[:, 0]),
            out("w_sq_v", w_sq_v), out("b_sq_v", None if w_sq_v is None else w_sq_v[:, 0]),
            out("w_sq_s", w_sq_s), out("b_sq_s", None if w_sq_s is None else w_sq_s[:, 0]),
            out("w_v", wv_), out("b_v", None if wv_ is None else wv_[:, 0]),
            None if share else out("w_s", ws_), None if share else out("b_s", None if ws_ is None else ws_[:, 0]),
            None)


class MMTM_mitigate(nn.Module):
    """Reference-compatible MMTM module (src/balanced_mmtm.py:15-154)."""

    def __init__(self, dim_visual, dim_skeleton, ratio, device=0, SEonly=False, shareweight=False):
        super().__init__()
        dim = dim_visual + dim_skeleton
        dim_out = int(2 * dim / ratio)
        self.SEonly = SEonly
        self.shareweight = shareweight
        dev = torch.device(f"cuda:{device}" if isinstance(device, int) else device)
        if dev.type == "cuda" and not torch.cuda.is_available():
            dev = torch.device("cpu")  # moved to the activations' device at first forward
        # plain attributes (not buffers), like the reference: not in state_dict
        self.running_avg_weight_visual = torch.zeros(dim_visual, device=dev)
        self.running_avg_weight_skeleton = torch.zeros(dim_visual, device=dev)
        self.step = 0
        if SEonly:
            self.fc_squeeze_visual = nn.Linear(dim_visual, dim_out)
            self.fc_squeeze_skeleton = nn.Linear(dim_skeleton, dim_out)
        else:
            self.fc_squeeze = nn.Linear(dim, dim_out)
        if shareweight:
            assert dim_visual == dim_skeleton
            self.fc_excite = nn.Linear(dim_out, dim_visual)
        else:
            self.fc_visual = nn.Linear(dim_out, dim_visual)
            self.fc_skeleton = nn.Linear(dim_out, dim_skeleton)
        self.relu = nn.ReLU()
        self.sigmoid = nn.Sigmoid()
        # data-parallel training needs every parameter to get a gradient every step:
        # when set, a curated branch receives zeros instead of None (identical SGD
        # update with momentum = weight_decay = 0, the reference's configs)
        self.zero_grads_for_curated = False
        # set by the engine's on-device gate: a device gm_gate_state whose flags replace
        # the curation_mode / caring_modality arguments
        self.device_gate = None
        # True: host flags drive the same select/mask kernels as the device gate (the
        # test that pins the device gate against the host gate bit for bit)
        self.mask_curation = False

    def _gate_for(self, curation_mode, caring_modality, dev):
        if self.device_gate is not None or not self.mask_curation:
            return self.device_gate
        st = L.GateState()
        st.curation_mode = int(bool(curation_mode))
        st.caring = -1 if caring_modality is None else int(caring_modality)
        return torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8).to(dev)

    def _lin(self, name):
        m = getattr(self, name, None)
        return (None, None) if m is None else (m.weight, m.bias)

    def forward(self, visual, skeleton, return_scale=False, return_squeezed_mps=False,
                turnoff_cross_modal_flow=False, average_squeezemaps=None, curation_mode=False,
                caring_modality=0):
        ops._dev_check(visual, skeleton)
        if visual.dtype not in ops._DT or skeleton.dtype != visual.dtype:
            raise L.GreedyMMLError(f"MMTM activations must be fp32 or bf16 (got {visual.dtype}, "
                                   f"{skeleton.dtype})")
        lay = ops.act_layout(visual)
        if lay is None:
            lay = L.GM_NCHW
        visual = ops.as_layout(visual, lay)
        skeleton = ops.as_layout(skeleton, lay)
        cfg, prm = self._site(visual.device, lay, return_squeezed_mps, turnoff_cross_modal_flow, average_squeezemaps,
                              curation_mode, caring_modality)
        yv, ys, e_v, e_s, sq = _MMTMFunction.apply(visual, skeleton, *prm, cfg)
        return (yv, ys) + self._record(e_v, e_s, sq, visual.shape[1], return_scale, return_squeezed_mps)

    def forward_stacked(self, X, return_scale=False, return_squeezed_mps=False, turnoff_cross_modal_flow=False,
                        average_squeezemaps=None, curation_mode=False, caring_modality=0):
        """forward() on the view-batched trunk's stacked activation X = [visual; skeleton]
        ([2B, C, H, W] channels_last, vtrunk.py): returns (Y stacked, scales, squeeze_array)."""
        if X.dtype not in ops._DT or X.shape[0] % 2 or not X.is_cuda:
            raise L.GreedyMMLError("MMTM stacked: fp32/bf16 HIP activations with an even batch")
        lay = ops.act_layout(X)
        if lay is None:
            lay = L.GM_NCHW
        X = ops.as_layout(X, lay)
        cfg, prm = self._site(X.device, lay, return_squeezed_mps, turnoff_cross_modal_flow, average_squeezemaps,
                              curation_mode, caring_modality)
        Y, e_v, e_s, sq = _MMTMStackedFn.apply(X, *prm, cfg)
        return (Y,) + self._record(e_v, e_s, sq, X.shape[1], return_scale, return_squeezed_mps)

    def _site(self, dev, lay, return_squeezed_mps, turnoff_cross_modal_flow, average_squeezemaps, curation_mode,
              caring_modality):
        """(cfg, parameters) of one site call: mode, running-average state, gate, curation."""
        if self.SEonly:
            mode = SEONLY
        elif turnoff_cross_modal_flow:
            mode = TURNOFF
        else:
            mode = NORMAL
        if return_squeezed_mps and mode != NORMAL:
            # reference: `squeeze_array` is only bound on the normal path
            raise UnboundLocalError("local variable 'squeeze_array' referenced before assignment")
        self.running_avg_weight_visual = _state_f32(self.running_avg_weight_visual, dev)
        self.running_avg_weight_skeleton = _state_f32(self.running_avg_weight_skeleton, dev)
        if self.running_avg_weight_skeleton.data_ptr() == self.running_avg_weight_visual.data_ptr():
            self.running_avg_weight_skeleton = self.running_avg_weight_skeleton.clone()
        step_dev = _step_counter(self, dev)
        cfg = dict(layout=lay, mode=mode, share=self.shareweight, step_dev=step_dev,
                   ra_v=self.running_avg_weight_visual,
                   ra_s=self.running_avg_weight_skeleton,
                   curation=bool(curation_mode), caring=caring_modality,
                   zero_curated=self.zero_grads_for_curated,
                   gate=self._gate_for(curation_mode, caring_modality, dev) if mode == NORMAL else None)
        if mode == TURNOFF:
            cfg["avg_v"] = _as_f32(average_squeezemaps[0], dev)
            cfg["avg_s"] = _as_f32(average_squeezemaps[1], dev)
        w_sq, b_sq = self._lin("fc_squeeze")
        w_sq_v, b_sq_v = self._lin("fc_squeeze_visual")
        w_sq_s, b_sq_s = self._lin("fc_squeeze_skeleton")
        if self.shareweight:
            w_v, b_v = self._lin("fc_excite")
            w_s = b_s = None
        else:
            w_v, b_v = self._lin("fc_visual")
            w_s, b_s = self._lin("fc_skeleton")
        return cfg, (w_sq, b_sq, w_sq_v, b_sq_v, w_sq_s, b_sq_s, w_v, b_v, w_s, b_s)

    def _record(self, e_v, e_s, sq, C1, return_scale, return_squeezed_mps):
        self.step += 1
        self._step_mirror = self.step
        scales = [e_v.cpu(), e_s.cpu()] if return_scale else None
        squeeze_array = None
        if return_squeezed_mps:
            squeeze_array = [sq[:, :C1].cpu(), sq[:, C1:].cpu()]
        return scales, squeeze_array


def get_mmtm_outputs(eval_save_path, mmtm_recorded, key):
    """Reference src/balanced_mmtm.py:157-176 (host-side, numpy)."""
    from .cur import mmtm_outputs
    return mmtm_outputs(eval_save_path, mmtm_recorded, key)


def get_rescale_weights(eval_save_path, training_save_path, key="test_squeezedmaps_array_list",
                        validation=False, starting_mmtmindice=1, mmtmpositions=4, device=None):
    """Reference src/balanced_mmtm.py:179-206."""
    from .cur import rescale_weights
    return rescale_weights(eval_save_path, training_save_path, key, validation,
                           starting_mmtmindice, mmtmpositions, device)
