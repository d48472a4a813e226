"""N-modality MMTM fusion (configs C4 = 4 ResNet-18 modalities,
C5 = 12 ResNet-50 views).

The reference's MMTM (src/balanced_mmtm.py:15-154) is hard-wired to two
modalities.  `MMTM_N(dims, ratio)` generalises its NORMAL, curation and
turn-off paths to N >= 2 modalities:

    sq    = [GAP(X_0) | ... | GAP(X_{N-1})]                      [B, sum C]
    z     = relu(fc_squeeze(sq))                                  [B, dim_out]
    e_i   = sigmoid(fc_excite[i](z))                              [B, C_i]
    Y_i   = X_i * e_i        (curation: e_caring <- running average)

Documented build decisions (no reference oracle beyond N = 2):

* dim_out = int(4 * sum(C) / (N * ratio)): the reference's int(2 * (Cv+Cs) /
  ratio) at N = 2, independent of N otherwise (the literal rule would give a
  24576 -> 12288 joint FC, 302 M weights per site, at C5's layer 4);
* running averages: `ra_source="first"` (default) updates every modality's
  average from modality 0's batch-mean scale, which at N = 2 is the reference's
  quirk (:113-116); `ra_source="own"` uses each modality's own scale;
* turn-off mode: modality i's joint-FC input is its own squeeze in its own
  segment and the dataset-average squeezes elsewhere (reference :72-91 at N = 2).

At N = 2 with the reference-compatible weights this is numerically the
reference's MMTM_mitigate (tests/test_gpu_mmtm_n.py checks it against the
same golden fixtures).  All arithmetic runs in libgreedymml_hip.so.
"""
import torch
import torch.nn as nn

from . import _lib as L
from . import ops
from .gradsink import sink_done, sink_target
from .ops import ONES, Op


def dim_out_rule(dims, ratio):
    return int(4 * sum(dims) / (len(dims) * ratio))


class _MMTMNFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, w_sq, b_sq, *rest):
        N = cfg["N"]
        ctx.gidx = (1, 2, 3 + N, 3 + 2 * N)  # needs_input_grad index of w_sq, b_sq, w_e[0], b_e[0]
        return _mmtmn_forward(ctx, cfg, w_sq, b_sq, list(rest[:N]), list(rest[N:2 * N]), list(rest[2 * N:3 * N]))

    @staticmethod
    def backward(ctx, *grads):
        return _mmtmn_backward(ctx, grads)


class _MMTMNStackedFn(torch.autograd.Function):
    """The same site over the view-batched trunk's stacked activation X ([N*B, C, H, W],
    view i = rows i*B..): Y is written as one stacked tensor and backward returns one
    stacked dX - no per-view slice gradients (autograd would zero-fill a full-size tensor
    per view) and no concatenation copies."""

    @staticmethod
    def forward(ctx, cfg, w_sq, b_sq, X, *rest):
        N = cfg["N"]
        B = X.shape[0] // N
        Y = torch.empty_like(X)
        ctx.gidx = (1, 2, 4, 4 + N)
        outs = _mmtmn_forward(ctx, cfg, w_sq, b_sq, [X[i * B:(i + 1) * B] for i in range(N)], list(rest[:N]),
                              list(rest[N:2 * N]), ys=[Y[i * B:(i + 1) * B] for i in range(N)])
        ctx.stacked_shape = (B, X.shape, X.dtype)
        return (Y,) + tuple(outs[N:])

    @staticmethod
    def backward(ctx, gY, *_rest):
        B, shape, dtype = ctx.stacked_shape
        N = ctx.meta[0]
        xv = ctx.saved_tensors[2]
        fmt = torch.channels_last if xv.is_contiguous(memory_format=torch.channels_last) else torch.contiguous_format
        dX = torch.empty(shape, device=xv.device, dtype=dtype, memory_format=fmt)
        grads = [None] * N if gY is None else [gY[i * B:(i + 1) * B] for i in range(N)]
        res = _mmtmn_backward(ctx, grads, dxs=[dX[i * B:(i + 1) * B] for i in range(N)])
        # res: (None, g_w_sq, g_b_sq, *dxs, *g_w_e, *g_b_e) -> (cfg, w_sq, b_sq, X, *w_e, *b_e)
        return (None, res[1], res[2], dX) + tuple(res[3 + N:])


def _mmtmn_forward(ctx, cfg, w_sq, b_sq, xs, w_e, b_e, ys=None):
    # no zero-filled gradients for the non-differentiable side outputs (the N excitations and
    # the squeeze): autograd otherwise materialises them, 3 x (N + 1) fills per C5 step
    ctx.set_materialize_grads(False)
    N = cfg["N"]
    dev = xs[0].device
    B = xs[0].shape[0]
    Cs = [x.shape[1] for x in xs]
    HWs = [x[0, 0].numel() for x in xs]
    offs = [sum(Cs[:i]) for i in range(N)]
    CT = sum(Cs)
    lay, dt = cfg["layout"], ops._DT[xs[0].dtype]
    f32 = dict(device=dev, dtype=torch.float32)
    Cz = w_sq.shape[0]
    sq = torch.empty(B, CT, **f32)
    ops.spatial_reduce([dict(x=xs[i], C=Cs[i], HW=HWs[i], out=sq, out_off=offs[i], ld_out=CT,
                             scale=1.0 / HWs[i]) for i in range(N)], B, dt, lay, dev)
    turnoff = cfg["turnoff"]
    if not turnoff:
        z = torch.empty(B, Cz, **f32)
        ops.gemm([dict(M=B, N=Cz, segs=[(CT, Op(sq, CT, 1), Op(w_sq, 1, CT))], C=z, ld_c=Cz,
                       bias=b_sq, act=1)], dev)
        zs = [z] * N
        ins = None
    else:
        avg = cfg["avg"]  # [CT] fp32: concatenated dataset-average squeezes
        ins, zs = [], []
        for i in range(N):
            inp = avg.view(1, CT).repeat(B, 1)
            inp[:, offs[i]:offs[i] + Cs[i]].copy_(sq[:, offs[i]:offs[i] + Cs[i]])
            ins.append(inp)
            zs.append(torch.empty(B, Cz, **f32))
        ops.gemm([dict(M=B, N=Cz, segs=[(CT, Op(ins[i], CT, 1), Op(w_sq, 1, CT))], C=zs[i], ld_c=Cz,
                       bias=b_sq, act=1) for i in range(N)], dev)
    es = [torch.empty(B, Cs[i], **f32) for i in range(N)]
    ops.gemm([dict(M=B, N=Cs[i], segs=[(Cz, Op(zs[i], Cz, 1), Op(w_e[i], 1, Cz))], C=es[i], ld_c=Cs[i],
                   bias=b_e[i], act=2) for i in range(N)], dev)
    # running averages (in place) + device step counter; reference quirk at N=2:
    # every average follows modality 0's scale
    ra = cfg["ra"]
    if cfg["ra_source"] == "first":
        pairs = [(i, min(i + 1, N - 1)) for i in range(0, N, 2)]
        for k, (i, j) in enumerate(pairs):
            ops.running_avg_dev(es[0], ra[i], ra[j], cfg["step_dev"], increment=k == len(pairs) - 1)
    else:
        for i in range(N):
            ops.running_avg_dev(es[i], ra[i], ra[i], cfg["step_dev"], increment=i == N - 1)
    ra_new = ra
    # on-device gate (engine, N branches): the flags live in device memory; the channel scale
    # reads the substituted modality's running average in place of its rows and backward
    # zeroes its excitation gradient inside the squeeze-backward launch (gm_mmtm_*_gated_n)
    gate = cfg.get("gate")
    caring = cfg["caring"] if (cfg["curation"] and gate is None) else None
    scl = [(es[i], Cs[i]) if i != caring else (ra_new[i], 0) for i in range(N)]
    if ys is None:
        ys = [torch.empty_like(x) for x in xs]
    ops.channel_scale([dict(x=xs[i], y=ys[i], C=Cs[i], HW=HWs[i], s=scl[i][0], ld_s=scl[i][1])
                       for i in range(N)], B, dt, lay, dev, gate=gate,
                      alt=None if gate is None else list(ra_new), mods=None if gate is None else list(range(N)))
    ctx.save_for_backward(sq, w_sq, *xs, *zs, *es, *w_e, *[s for s, _ in scl], *(ins or []))
    ctx.meta = (N, B, Cs, HWs, offs, CT, Cz, lay, dt, turnoff, caring, [ld for _, ld in scl],
                cfg["zero_curated"], gate, list(ra_new))
    ctx.mark_non_differentiable(*es, sq)
    ctx.prm = (w_sq, b_sq, list(w_e), list(b_e))  # the leaves, for in-place delivery (gradsink)
    return (*ys, *es, sq)


def _mmtmn_backward(ctx, grads, dxs=None):
    N, B, Cs, HWs, offs, CT, Cz, lay, dt, turnoff, caring, lds, zero_curated, gate, ra = ctx.meta
    sv = ctx.saved_tensors
    sq, w_sq = sv[0], sv[1]
    xs = list(sv[2:2 + N])
    zs = list(sv[2 + N:2 + 2 * N])
    es = list(sv[2 + 2 * N:2 + 3 * N])
    w_e = list(sv[2 + 3 * N:2 + 4 * N])
    scl = list(sv[2 + 4 * N:2 + 5 * N])
    ins = list(sv[2 + 5 * N:2 + 6 * N]) if turnoff else None
    dev = xs[0].device
    f32 = dict(device=dev, dtype=torch.float32)
    gy = []
    for i in range(N):
        g = grads[i]
        g = torch.zeros_like(xs[i]) if g is None else ops.as_layout(g.to(xs[i].dtype), lay)
        gy.append(g)
    live = [i for i in range(N) if i != caring]
    da = {i: torch.empty(B, Cs[i], **f32) for i in live}
    ops.spatial_reduce([dict(x=xs[i], dy=gy[i], C=Cs[i], HW=HWs[i], out=da[i], ld_out=Cs[i], e=es[i],
                             ld_e=Cs[i]) for i in live], B, dt, lay, dev, gate=gate,
                       mods=None if gate is None else live)
    # parameter gradients: written by the GEMMs straight into the engine's flat gradient
    # buffer when the parameter is sink-managed (no AccumulateGrad fill + add per tensor)
    p_wsq, p_bsq, p_we, p_be = ctx.prm
    i_wsq, i_bsq, i_we, i_be = ctx.gidx
    sunk = []

    def gbuf(prm, idx, *shape):
        tgt = sink_target(prm) if ctx.needs_input_grad[idx] else None
        if tgt is None:
            return torch.empty(*shape, **f32), 0
        t, acc = tgt
        if not t.is_contiguous() or tuple(t.shape) != shape:
            raise RuntimeError(f"MMTM_N: in-place gradient buffer must be a contiguous {shape}")
        sunk.append((prm, t))
        return t, int(acc)

    gw = {}
    gb = {}
    probs = []
    for i in live:
        gw[i], acc_w = gbuf(p_we[i], i_we + i, Cs[i], Cz)
        gb[i], acc_b = gbuf(p_be[i], i_be + i, Cs[i])
        probs += [dict(M=Cs[i], N=Cz, segs=[(B, Op(da[i], 1, Cs[i]), Op(zs[i], Cz, 1))], C=gw[i], ld_c=Cz,
                       accumulate=acc_w),
                  dict(M=1, N=Cs[i], segs=[(B, ONES, Op(da[i], Cs[i], 1))], C=gb[i], ld_c=Cs[i],
                       accumulate=acc_b)]
    ops.gemm(probs, dev)
    # dz: NORMAL sums every live modality's contribution (2 K-segments per launch,
    # later launches accumulate; the relu mask is linear so it applies per launch)
    g_sq_w = g_sq_b = None
    dsq = None
    if live:
        if not turnoff:
            dz = torch.empty(B, Cz, **f32)
            for n, k in enumerate(range(0, len(live), 2)):
                segs = [(Cs[i], Op(da[i], Cs[i], 1), Op(w_e[i], Cz, 1)) for i in live[k:k + 2]]
                ops.gemm([dict(M=B, N=Cz, segs=segs, C=dz, ld_c=Cz, mask=zs[0], ld_mask=Cz,
                               accumulate=int(n > 0))], dev)
            dsq = torch.empty(B, CT, **f32)
            g_sq_w, acc_w = gbuf(p_wsq, i_wsq, Cz, CT)
            g_sq_b, acc_b = gbuf(p_bsq, i_bsq, Cz)
            ops.gemm([dict(M=Cz, N=CT, segs=[(B, Op(dz, 1, Cz), Op(sq, CT, 1))], C=g_sq_w, ld_c=CT,
                           accumulate=acc_w),
                      dict(M=1, N=Cz, segs=[(B, ONES, Op(dz, Cz, 1))], C=g_sq_b, ld_c=Cz, accumulate=acc_b),
                      dict(M=B, N=CT, segs=[(Cz, Op(dz, Cz, 1), Op(w_sq, CT, 1))], C=dsq, ld_c=CT)], dev)
        else:
            dzs = {i: torch.empty(B, Cz, **f32) for i in live}
            ops.gemm([dict(M=B, N=Cz, segs=[(Cs[i], Op(da[i], Cs[i], 1), Op(w_e[i], Cz, 1))], C=dzs[i],
                           ld_c=Cz, mask=zs[i], ld_mask=Cz) for i in live], dev)
            g_sq_w, acc_w = gbuf(p_wsq, i_wsq, Cz, CT)
            g_sq_b, acc_b = gbuf(p_bsq, i_bsq, Cz)
            for n, k in enumerate(range(0, len(live), 2)):
                grp = live[k:k + 2]
                ops.gemm([dict(M=Cz, N=CT, segs=[(B, Op(dzs[i], 1, Cz), Op(ins[i], CT, 1)) for i in grp],
                               C=g_sq_w, ld_c=CT, accumulate=int(n > 0) | acc_w),
                          dict(M=1, N=Cz, segs=[(B, ONES, Op(dzs[i], Cz, 1)) for i in grp], C=g_sq_b,
                               ld_c=Cz, accumulate=int(n > 0) | acc_b)], dev)
            dsq = torch.zeros(B, CT, **f32)
            ops.gemm([dict(M=B, N=Cs[i], segs=[(Cz, Op(dzs[i], Cz, 1), Op(w_sq, CT, 1, off=offs[i]))],
                           C=dsq, c_off=offs[i], ld_c=CT) for i in live], dev)
    if dxs is None:
        dxs = [torch.empty_like(x) for x in xs]
    probs = []
    for i in range(N):
        p = dict(x=gy[i], y=dxs[i], C=Cs[i], HW=HWs[i], s=scl[i], ld_s=lds[i])
        if dsq is not None:
            p.update(a=dsq, a_off=offs[i], ld_a=CT, alpha=1.0 / HWs[i])
        probs.append(p)
    ops.channel_scale(probs, B, dt, lay, dev, gate=gate, alt=None if gate is None else ra,
                      mods=None if gate is None else list(range(N)))
    for prm, _ in sunk:  # delivered in place: fire the engine's per-parameter hook
        sink_done(prm)
    sunk_ids = {id(t) for _, t in sunk}

    def z_or_none(t, like):
        if t is not None:
            return None if id(t) in sunk_ids else t
        return torch.zeros_like(like) if zero_curated else None
    out_we = [z_or_none(gw.get(i), w_e[i]) for i in range(N)]
    out_be = [z_or_none(gb.get(i), w_e[i][:, 0]) for i in range(N)]
    return (None, z_or_none(g_sq_w, w_sq), z_or_none(g_sq_b, w_sq[:, 0]), *dxs, *out_we, *out_be)


class MMTM_N(nn.Module):
    """N-modality MMTM (see module doc).  Parameters: fc_squeeze, fc_excite.{i}."""

    def __init__(self, dims, ratio, ra_source="first"):
        super().__init__()
        dims = list(dims)
        if len(dims) < 2:
            raise ValueError("MMTM_N needs at least two modalities")
        if ra_source not in ("first", "own"):
            raise ValueError("ra_source must be 'first' or 'own'")
        self.dims = dims
        self.N = len(dims)
        self.ra_source = ra_source
        if ra_source == "first" and len(set(dims)) != 1:
            raise ValueError("ra_source='first' needs equal channel counts")
        dim_out = dim_out_rule(dims, ratio)
        self.fc_squeeze = nn.Linear(sum(dims), dim_out)
        self.fc_excite = nn.ModuleList([nn.Linear(dim_out, d) for d in dims])
        self.running_avg = [torch.zeros(d) for d in dims]
        self.step = 0
        self.zero_grads_for_curated = False
        # set by the engine's on-device gate: a device gm_gate_state_n whose flags replace
        # the curation_mode / caring_modality arguments
        self.device_gate = None
        # True: host flags drive the same gated kernels as the device gate (the test that
        # pins the N-branch device gate against the host gate bit for bit)
        self.mask_curation = False

    def _gate_for(self, curation_mode, caring_modality, dev):
        if self.device_gate is not None or not self.mask_curation:
            return self.device_gate
        st = L.GateStateN()
        st.curation_mode = int(bool(curation_mode))
        st.caring = int(caring_modality) if curation_mode else -1
        st.nb = self.N
        return torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8).to(dev)

    def forward_stacked(self, X, return_scale=False, return_squeezed_mps=False, turnoff_cross_modal_flow=False,
                        average_squeezemaps=None, curation_mode=False, caring_modality=0):
        """forward() over the view-batched trunk's stacked activation X = [x_0; ...; x_{N-1}]
        ([N*B, C, H, W] channels_last, vtrunk.py): returns (Y stacked, scales, squeeze)."""
        if X.shape[0] % self.N or not X.is_cuda or X.dtype not in ops._DT:
            raise L.GreedyMMLError("MMTM_N stacked: fp32/bf16 HIP activations with a batch divisible by N")
        lay = ops.act_layout(X)
        if lay is None:
            lay = L.GM_NCHW
        X = ops.as_layout(X, lay)
        cfg, w_e, b_e = self._site(X.device, lay, return_squeezed_mps, turnoff_cross_modal_flow, average_squeezemaps,
                                   curation_mode, caring_modality)
        outs = _MMTMNStackedFn.apply(cfg, self.fc_squeeze.weight, self.fc_squeeze.bias, X, *w_e, *b_e)
        return (outs[0],) + self._record(list(outs[1:1 + self.N]), outs[1 + self.N], return_scale,
                                         return_squeezed_mps)

    def _site(self, dev, lay, return_squeezed_mps, turnoff_cross_modal_flow, average_squeezemaps, curation_mode,
              caring_modality):
        from .balanced_mmtm import _state_f32, _step_counter
        self.running_avg = [_state_f32(r, dev) for r in self.running_avg]
        if curation_mode and not (0 <= int(caring_modality) < self.N):
            raise ValueError(f"caring_modality must be in [0, {self.N})")
        cfg = dict(N=self.N, layout=lay, turnoff=bool(turnoff_cross_modal_flow), step_dev=_step_counter(self, dev),
                   ra=self.running_avg, ra_source=self.ra_source,
                   curation=bool(curation_mode), caring=int(caring_modality) if curation_mode else None,
                   zero_curated=self.zero_grads_for_curated,
                   gate=None if turnoff_cross_modal_flow else self._gate_for(curation_mode, caring_modality, dev))
        if turnoff_cross_modal_flow:
            if return_squeezed_mps:
                raise UnboundLocalError("local variable 'squeeze_array' referenced before assignment")
            cfg["avg"] = torch.cat([torch.as_tensor(a).to(device=dev, dtype=torch.float32).reshape(-1)
                                    for a in average_squeezemaps]).contiguous()
        return cfg, [m.weight for m in self.fc_excite], [m.bias for m in self.fc_excite]

    def _record(self, es, sq, return_scale, return_squeezed_mps):
        self.step += 1
        self._step_mirror = self.step
        scales = [e.cpu() for e in es] if return_scale else None
        squeeze = None
        if return_squeezed_mps:
            squeeze = [t.cpu() for t in torch.split(sq, self.dims, dim=1)]
        return scales, squeeze

    def forward(self, xs, return_scale=False, return_squeezed_mps=False, turnoff_cross_modal_flow=False,
                average_squeezemaps=None, curation_mode=False, caring_modality=0):
        xs = list(xs)
        if len(xs) != self.N:
            raise ValueError(f"expected {self.N} modalities, got {len(xs)}")
        ops._dev_check(*xs)
        dt = xs[0].dtype
        if dt not in ops._DT or any(x.dtype != dt for x in xs):
            raise L.GreedyMMLError("MMTM_N activations must all be fp32 or all bf16")
        dev = xs[0].device
        lay = ops.act_layout(xs[0])
        if lay is None:
            lay = L.GM_NCHW
        xs = [ops.as_layout(x, lay) for x in xs]
        cfg, w_e, b_e = self._site(dev, lay, return_squeezed_mps, turnoff_cross_modal_flow, average_squeezemaps,
                                   curation_mode, caring_modality)
        outs = _MMTMNFunction.apply(cfg, self.fc_squeeze.weight, self.fc_squeeze.bias, *xs, *w_e, *b_e)
        ys, es, sq = list(outs[:self.N]), list(outs[self.N:2 * self.N]), outs[2 * self.N]
        scales, squeeze = self._record(es, sq, return_scale, return_squeezed_mps)
        return ys, scales, squeeze
