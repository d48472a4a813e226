"""Thin tensor-level wrappers over the C ABI (include/greedymml.h).

Every function takes device tensors, launches on the current HIP stream of
their device and raises GreedyMMLError on failure.  No CPU path exists: a
non-HIP tensor is an error.
"""
import ctypes

import torch

from . import _lib as L

_DT = {torch.float32: L.GM_F32, torch.bfloat16: L.GM_BF16}


def _dev_check(*ts):
    for t in ts:
        if t is not None and (not t.is_cuda):
            raise L.GreedyMMLError(
                "greedy_multimodal_learning_amd ops run on HIP devices only (got a "
                f"{t.device} tensor); there is no CPU fallback")


def act_layout(x):
    """GM_NCHW / GM_NHWC for a 4-D (or [B,C,...]) activation, or None if neither."""
    if x.dim() == 4 and not x.is_contiguous() and x.is_contiguous(memory_format=torch.channels_last):
        return L.GM_NHWC
    if x.is_contiguous():
        return L.GM_NCHW
    return None


def as_layout(x, layout):
    if layout == L.GM_NHWC:
        return x.contiguous(memory_format=torch.channels_last)
    return x.contiguous()


MAX_REDUCE, MAX_SCALE, MAX_GEMM = 4, 4, 6  # problems per launch (include/greedymml.h)


def spatial_reduce(probs, B, dtype, layout, device, gate=None, mods=None):
    """probs: list of dict(x, dy, out, ld_out, e, ld_e, C, HW, scale, out_off) -> launches.
    gate (device gm_gate_state): problems 0 / 1 are the two modalities and the substituted
    one's outputs are zeroed in the same launch (gm_mmtm_spatial_reduce_gated); with
    mods (modality id per problem, N-modality form) any number of problems
    (gm_mmtm_spatial_reduce_gated_n, MAX_REDUCE per launch)."""
    if gate is not None and mods is None:
        assert 2 <= len(probs) <= MAX_REDUCE
    if len(probs) > MAX_REDUCE:
        for i in range(0, len(probs), MAX_REDUCE):
            spatial_reduce(probs[i:i + MAX_REDUCE], B, dtype, layout, device, gate=gate,
                           mods=None if mods is None else mods[i:i + MAX_REDUCE])
        return
    lib = L.load()
    items = []
    for p in probs:
        out = p["out"]
        items.append(L.SpatialReduce(
            L.ptr(p["x"]), L.ptr(p.get("dy")), p["C"], p["HW"],
            out.data_ptr() + 4 * p.get("out_off", 0), p["ld_out"],
            L.ptr(p.get("e")) + 4 * p.get("e_off", 0) if p.get("e") is not None else 0,
            p.get("ld_e", 0), p.get("scale", 1.0)))
    a = L.arr(L.SpatialReduce, items)
    need = lib.gm_spatial_reduce_scratch(a, len(items), B, dtype, layout)
    scratch = torch.empty(max(need, 16), dtype=torch.uint8, device=device) if need else None
    if gate is not None and mods is not None:
        m = (ctypes.c_int * len(items))(*[int(v) for v in mods])
        L.check(lib.gm_mmtm_spatial_reduce_gated_n(a, len(items), B, dtype, layout, gate.data_ptr(), m,
                                                   L.ptr(scratch), need, L.stream_of(device)),
                "gm_mmtm_spatial_reduce_gated_n")
        return
    if gate is not None:
        L.check(lib.gm_mmtm_spatial_reduce_gated(a, len(items), B, dtype, layout, gate.data_ptr(), L.ptr(scratch),
                                                 need, L.stream_of(device)), "gm_mmtm_spatial_reduce_gated")
        return
    L.check(lib.gm_mmtm_spatial_reduce(a, len(items), B, dtype, layout, L.ptr(scratch), need,
                                       L.stream_of(device)), "gm_mmtm_spatial_reduce")


def channel_scale(probs, B, dtype, layout, device, gate=None, alt=None, mods=None):
    """probs: list of dict(x, y, C, HW, s, s_off, ld_s, a, a_off, ld_a, alpha).
    gate (device gm_gate_state) + alt (two fp32 rows): problems 0 / 1 are the two
    modalities and the substituted one scales by its alt row (gm_mmtm_channel_scale_gated);
    with mods (modality id per problem) alt holds one row per problem and any number of
    problems is allowed (gm_mmtm_channel_scale_gated_n, MAX_SCALE per launch)."""
    if gate is not None:
        assert alt is not None
        if mods is None:
            assert 2 <= len(probs) <= MAX_SCALE
        else:
            assert len(mods) == len(alt) == len(probs)
    if len(probs) > MAX_SCALE:
        for i in range(0, len(probs), MAX_SCALE):
            sl = slice(i, i + MAX_SCALE)
            channel_scale(probs[sl], B, dtype, layout, device, gate=gate,
                          alt=None if mods is None else alt[sl], mods=None if mods is None else mods[sl])
        return
    lib = L.load()
    items = []
    for p in probs:
        a = p.get("a")
        items.append(L.ChannelScale(
            L.ptr(p["x"]), L.ptr(p["y"]), p["C"], p["HW"],
            p["s"].data_ptr() + 4 * p.get("s_off", 0), p["ld_s"],
            (a.data_ptr() + 4 * p.get("a_off", 0)) if a is not None else 0, p.get("ld_a", 0),
            p.get("alpha", 0.0)))
    arr = L.arr(L.ChannelScale, items)
    if gate is not None and mods is not None:
        m = (ctypes.c_int * len(items))(*[int(v) for v in mods])
        rows = (ctypes.c_void_p * len(items))(*[r.data_ptr() for r in alt])
        L.check(lib.gm_mmtm_channel_scale_gated_n(arr, len(items), B, dtype, layout, gate.data_ptr(), m, rows,
                                                  L.stream_of(device)), "gm_mmtm_channel_scale_gated_n")
        return
    if gate is not None:
        L.check(lib.gm_mmtm_channel_scale_gated(arr, len(items), B, dtype, layout, gate.data_ptr(), alt[0].data_ptr(),
                                                alt[1].data_ptr(), L.stream_of(device)),
                "gm_mmtm_channel_scale_gated")
        return
    L.check(lib.gm_mmtm_channel_scale(arr, len(items), B, dtype, layout, L.stream_of(device)),
            "gm_mmtm_channel_scale")


class Op:
    """A strided fp32 operand view: element (i, j) at base[off + i*ld0 + j*ld1]."""
    __slots__ = ("t", "off", "ld0", "ld1")

    def __init__(self, t, ld0, ld1, off=0):
        self.t, self.ld0, self.ld1, self.off = t, ld0, ld1, off

    def c(self):
        return L.Operand(0 if self.t is None else self.t.data_ptr() + 4 * self.off, self.ld0, self.ld1)


ONES = Op(None, 0, 0)


def gemm(problems, device):
    """problems: list of dict(M, N, segs=[(K, Op A, Op B)], C, c_off, ld_c, bias, act, mask,
    ld_mask, accumulate). C[m,n] (+)= act(sum_seg A.B + bias) * (mask > 0).
    Problems must be independent (no problem reads another's output)."""
    if len(problems) > MAX_GEMM:
        for i in range(0, len(problems), MAX_GEMM):
            gemm(problems[i:i + MAX_GEMM], device)
        return
    lib = L.load()
    items = []
    for p in problems:
        segs = p["segs"]
        assert 1 <= len(segs) <= 2
        K = (L.c_int * 2)(*[s[0] for s in segs] + [0] * (2 - len(segs)))
        A = (L.Operand * 2)(*[s[1].c() for s in segs] + [L.Operand(0, 0, 0)] * (2 - len(segs)))
        Bm = (L.Operand * 2)(*[s[2].c() for s in segs] + [L.Operand(0, 0, 0)] * (2 - len(segs)))
        Ct = p["C"]
        items.append(L.Gemm(p["M"], p["N"], K, A, Bm, L.ptr(p.get("bias")), L.ptr(p.get("mask")),
                            p.get("ld_mask", 0), Ct.data_ptr() + 4 * p.get("c_off", 0), p["ld_c"],
                            p.get("act", 0), int(p.get("accumulate", 0))))
    arr = L.arr(L.Gemm, items)
    L.check(lib.gm_gemm_f32(arr, len(items), L.stream_of(device)), "gm_gemm_f32")


def running_avg(e_v, ra_v, ra_s, step):
    lib = L.load()
    B, C = e_v.shape
    nv, ns = torch.empty_like(ra_v), torch.empty_like(ra_s)
    L.check(lib.gm_mmtm_running_avg(e_v.data_ptr(), e_v.stride(0), B, C, ra_v.data_ptr(),
                                    ra_s.data_ptr(), nv.data_ptr(), ns.data_ptr(), int(step),
                                    L.stream_of(e_v.device)), "gm_mmtm_running_avg")
    return nv, ns


def running_avg_dev(e_v, ra_v, ra_s, step_dev, increment=True):
    """In-place running-average update with a device step counter (graph-capturable)."""
    lib = L.load()
    B, C = e_v.shape
    L.check(lib.gm_mmtm_running_avg_dev(e_v.data_ptr(), e_v.stride(0), B, C, ra_v.data_ptr(), ra_s.data_ptr(),
                                        step_dev.data_ptr(), int(increment), L.stream_of(e_v.device)),
            "gm_mmtm_running_avg_dev")


def linear(x, w, b=None, act=0):
    """y = act(x @ w.T + b) on the fp32 MFMA GEMM (x [M,K], w [N,K])."""
    _dev_check(x, w)
    x = x.float().contiguous()
    M, K = x.shape
    N = w.shape[0]
    y = torch.empty(M, N, device=x.device, dtype=torch.float32)
    gemm([dict(M=M, N=N, segs=[(K, Op(x, K, 1), Op(w, 1, K))], C=y, ld_c=N, bias=b, act=act)],
         x.device)
    return y
