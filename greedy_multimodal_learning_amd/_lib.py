"""ctypes binding of libgreedymml_hip.so (the C ABI in include/greedymml.h).

The library is loaded AFTER `import torch` so that it binds to PyTorch's HIP
runtime instance (same SONAME libamdhip64.so.7).  There is no fallback: if the
library is missing or fails to load, every op raises.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL: shared HIP runtime)

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "libgreedymml_hip.so")

GM_F32, GM_BF16 = 0, 1
GM_NCHW, GM_NHWC = 0, 1
ABI_VERSION = 3

c_int, c_float, c_void_p, c_size_t = ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t
c_float_p = ctypes.c_void_p  # device pointers are opaque


class SpatialReduce(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("dy", c_void_p), ("C", c_int), ("HW", c_int),
                ("out", c_void_p), ("ld_out", c_int), ("e", c_void_p), ("ld_e", c_int),
                ("scale", c_float)]


class ChannelScale(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("y", c_void_p), ("C", c_int), ("HW", c_int),
                ("s", c_void_p), ("ld_s", c_int), ("a", c_void_p), ("ld_a", c_int),
                ("alpha", c_float)]


class Operand(ctypes.Structure):
    _fields_ = [("ptr", c_void_p), ("ld0", c_int), ("ld1", c_int)]


class Gemm(ctypes.Structure):
    _fields_ = [("M", c_int), ("N", c_int), ("K", c_int * 2), ("A", Operand * 2),
                ("B", Operand * 2), ("bias", c_void_p), ("mask", c_void_p), ("ld_mask", c_int),
                ("C", c_void_p), ("ld_c", c_int), ("act", c_int), ("accumulate", c_int)]


class Tensor(ctypes.Structure):
    _fields_ = [("param", c_void_p), ("grad", c_void_p), ("n", ctypes.c_longlong),
                ("offset", ctypes.c_longlong), ("group_mask", ctypes.c_uint),
                ("pad", ctypes.c_uint)]


EXPORTS = {
    "gm_abi_version": (c_int, []),
    "gm_last_error": (ctypes.c_char_p, []),
    "gm_spatial_reduce_scratch": (c_size_t, [c_void_p, c_int, c_int, c_int, c_int]),
    "gm_mmtm_spatial_reduce": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_size_t,
                                       c_void_p]),
    "gm_mmtm_set_reduce_form": (c_int, [c_int, c_int]),
    "gm_mmtm_channel_scale": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "gm_gemm_f32": (c_int, [c_void_p, c_int, c_void_p]),
    "gm_gemm_set_form": (c_int, [c_int]),
    "gm_mmtm_running_avg": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_int, c_void_p]),
    "gm_mmtm_running_avg_dev": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                        c_void_p]),
    "gm_group_sumsq_scratch": (c_size_t, [ctypes.c_longlong]),
    "gm_group_sumsq": (c_int, [c_void_p, c_int, ctypes.c_longlong, c_int, c_float, c_float,
                               c_void_p, c_void_p, c_size_t, c_void_p]),
    "gm_group_sumsq_gate": (c_int, [c_void_p, c_int, ctypes.c_longlong, c_int, c_float, c_float,
                                    c_void_p, c_void_p, c_size_t, c_void_p, c_int, c_void_p]),
}

_lib = None


class GreedyMMLError(RuntimeError):
    pass


def load():
    """Load (once) and return the CDLL; raises if the HIP library is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GreedyMMLError(
            f"{LIB_PATH} not built: run `python -m greedy_multimodal_learning_amd.build` "
            "(no CPU fallback exists)")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
    for name, (res, args) in EXPORTS.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    v = lib.gm_abi_version()
    if v != ABI_VERSION:
        raise GreedyMMLError(f"ABI mismatch: library {v}, bindings {ABI_VERSION}")
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        msg = load().gm_last_error().decode(errors="replace")
        raise GreedyMMLError(f"{what} failed (rc={rc}): {msg}")


def ptr(t):
    """Device pointer of a tensor (0 for None)."""
    return 0 if t is None else t.data_ptr()


def stream_of(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def arr(struct_type, items):
    a = (struct_type * len(items))(*items)
    return a


class ConvDesc(ctypes.Structure):
    _fields_ = [("N", c_int), ("H", c_int), ("W", c_int), ("C", c_int), ("K", c_int),
                ("R", c_int), ("S", c_int), ("stride", c_int), ("pad", c_int)]


EXPORTS.update({
    "gm_conv2d_fwd_bf16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gm_conv2d_dgrad_bf16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gm_conv_weight_transpose_bf16": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "gm_conv2d_wgrad_scratch": (c_size_t, [c_void_p]),
    "gm_conv_weight_prep_bf16": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "gm_conv2d_wgrad_bf16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p,
                                     c_size_t, c_void_p]),
    "gm_wprep_tiles": (c_int, [c_int, c_int, c_int]),
    "gm_conv_weight_prep_multi_bf16": (c_int, [c_void_p, c_int, c_int, c_void_p]),
})


class ConvDescHW(ctypes.Structure):
    _fields_ = [("N", c_int), ("H", c_int), ("W", c_int), ("C", c_int), ("K", c_int), ("R", c_int), ("S", c_int),
                ("stride_h", c_int), ("stride_w", c_int), ("pad_h", c_int), ("pad_w", c_int)]


EXPORTS.update({
    "gm_conv2d_fwd_hw_bf16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gm_conv2d_splitk_ws_bytes": (c_size_t, [c_void_p, c_int]),
    "gm_conv2d_fwd_ex_bf16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "gm_conv2d_dgrad_ex_bf16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "gm_conv2d_dgrad_add_bf16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                         c_void_p]),
    "gm_conv2d_wgrad_hw_scratch": (c_size_t, [c_void_p]),
    # view groups: G views stacked along the batch, one weight per view
    "gm_conv2d_fwd_grouped_bf16": (c_int, [c_void_p, c_int, c_void_p, c_void_p, ctypes.c_longlong, c_void_p,
                                           c_void_p, c_size_t, c_void_p]),
    "gm_conv2d_dgrad_grouped_bf16": (c_int, [c_void_p, c_int, c_void_p, c_void_p, ctypes.c_longlong, c_void_p,
                                             c_void_p, c_void_p, c_size_t, c_void_p]),
    "gm_conv2d_dgrad_grouped_masked_bf16": (c_int, [c_void_p, c_int, c_void_p, c_void_p, ctypes.c_longlong,
                                                    c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "gm_conv2d_splitk_ws_bytes_grouped": (c_size_t, [c_void_p, c_int, c_int]),
    "gm_conv2d_wgrad_grouped_scratch": (c_size_t, [c_void_p, c_int]),
    "gm_conv2d_wgrad_grouped_bf16": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, ctypes.c_longlong,
                                             c_int, c_int, c_void_p, c_size_t, c_void_p]),
    "gm_conv2d_wgrad_hw_bf16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p,
                                        c_size_t, c_void_p]),
    "gm_stem_dw_crop": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "gm_conv2d_wgrad_stem_bn_ok": (c_int, [c_void_p, c_int]),
    "gm_conv2d_wgrad_stem_bn_grouped_bf16": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                                     ctypes.c_longlong, c_int, c_void_p, c_size_t, c_void_p]),
})


class StemBnSrc(ctypes.Structure):
    """gm_stem_bn_src: the stem BatchNorm + ReLU + max-pool backward's operands, for the stem
    weight gradient that forms its dy in the loader"""
    _fields_ = [("y", c_void_p), ("dy_pool", c_void_p), ("idx", c_void_p), ("fcoef", c_void_p),
                ("fcoef_gs", ctypes.c_longlong), ("bcoef", c_void_p), ("bcoef_gs", ctypes.c_longlong)]


class WPrep(ctypes.Structure):
    _fields_ = [("w", c_void_p), ("wb", c_void_p), ("wt", c_void_p), ("K", c_int), ("RS", c_int),
                ("C", c_int), ("Cp", c_int), ("tile_start", c_int), ("pad", c_int)]


class GateState(ctypes.Structure):
    _fields_ = [("curation_mode", c_int), ("caring", c_int), ("curation_step", c_int), ("unlock", c_int),
                ("window", c_int), ("n_curated", c_int), ("pad0", c_int), ("pad1", c_int),
                ("eps", ctypes.c_double), ("M", ctypes.c_double * 4), ("d_bdr", ctypes.c_double)]


GATE_MAX_BRANCHES = 16


class GateStateN(ctypes.Structure):
    """gm_gate_state_n: the N-branch on-device gate (same 32-byte prefix as GateState)."""
    _fields_ = [("curation_mode", c_int), ("caring", c_int), ("curation_step", c_int), ("unlock", c_int),
                ("window", c_int), ("n_curated", c_int), ("nb", c_int), ("pad0", c_int),
                ("eps", ctypes.c_double), ("M_bypass", ctypes.c_double * GATE_MAX_BRANCHES),
                ("M_main", ctypes.c_double * GATE_MAX_BRANCHES), ("bdr", ctypes.c_double * GATE_MAX_BRANCHES),
                ("d_bdr", ctypes.c_double)]


class StemPack(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("dtype", c_int), ("N", c_int), ("C0", c_int), ("H", c_int), ("W", c_int),
                ("pad", c_int), ("sn", ctypes.c_longlong), ("sc", ctypes.c_longlong), ("sh", ctypes.c_longlong),
                ("sw", ctypes.c_longlong), ("Hp", c_int), ("Wp", c_int), ("xp", c_void_p), ("w", c_void_p),
                ("K", c_int), ("R", c_int), ("S", c_int), ("wp", c_void_p), ("wk", ctypes.c_longlong),
                ("wc", ctypes.c_longlong), ("wr", ctypes.c_longlong), ("ws", ctypes.c_longlong)]


EXPORTS.update({
    "gm_gate_strong_step": (c_int, [c_void_p, c_void_p, c_void_p]),
    "gm_gate_strong_step_n": (c_int, [c_void_p, c_void_p, c_void_p]),
    "gm_mmtm_channel_scale_gated_n": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                              c_void_p]),
    "gm_mmtm_spatial_reduce_gated_n": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                               ctypes.c_size_t, c_void_p]),
    "gm_mmtm_select_scale": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                                     c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gm_mmtm_mask_rows": (c_int, [c_void_p, ctypes.c_longlong, c_void_p, c_void_p]),
    "gm_mmtm_mask_rows2": (c_int, [c_void_p, ctypes.c_longlong, c_void_p, ctypes.c_longlong, c_void_p, c_void_p]),
    "gm_mmtm_channel_scale_gated": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                            c_void_p]),
    "gm_mmtm_spatial_reduce_gated": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_size_t,
                                             c_void_p]),
    "gm_stem_pack_bf16": (c_int, [c_void_p, c_void_p]),
    "gm_stem_pack_grouped_bf16": (c_int, [c_void_p, c_int, c_void_p]),
    "gm_xent_fwd": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gm_xent_bwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
})


class BnFwd(ctypes.Structure):
    _fields_ = [("M", ctypes.c_longlong), ("C", c_int), ("relu", c_int), ("x", c_void_p),
                ("residual", c_void_p), ("y", c_void_p), ("gamma", c_void_p), ("beta", c_void_p),
                ("running_mean", c_void_p), ("running_var", c_void_p), ("momentum", c_float),
                ("eps", c_float), ("save_mean", c_void_p), ("save_invstd", c_void_p),
                ("num_batches_tracked", c_void_p), ("coef_out", c_void_p), ("relu_mask", c_void_p)]


class BnBwd(ctypes.Structure):
    _fields_ = [("M", ctypes.c_longlong), ("C", c_int), ("relu", c_int), ("dy", c_void_p),
                ("y", c_void_p), ("x", c_void_p), ("gamma", c_void_p), ("save_mean", c_void_p),
                ("save_invstd", c_void_p), ("dx", c_void_p), ("dres", c_void_p), ("dgamma", c_void_p),
                ("dbeta", c_void_p), ("accumulate", c_int), ("pad", c_int), ("fwd_coef", c_void_p),
                ("relu_mask", c_void_p)]


EXPORTS.update({
    "gm_bn_scratch": (c_size_t, [ctypes.c_longlong, c_int]),
    "gm_bn_fwd_train_bf16": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "gm_bn_fwd_stats_bf16": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "gm_bn_scratch_grouped": (c_size_t, [ctypes.c_longlong, c_int, c_int]),
    "gm_bn_fwd_train_grouped_bf16": (c_int, [c_void_p, c_int, c_void_p, c_size_t, c_void_p]),
    "gm_bn_bwd_grouped_bf16": (c_int, [c_void_p, c_int, c_void_p, c_size_t, c_void_p]),
    "gm_bn_fwd_stats_grouped_bf16": (c_int, [c_void_p, c_int, c_void_p, c_size_t, c_void_p]),
    "gm_bn_fwd_infer_bf16": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "gm_bn_bwd_bf16": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
})


class PoolDesc(ctypes.Structure):
    _fields_ = [("N", c_int), ("H", c_int), ("W", c_int), ("C", c_int), ("k", c_int), ("stride", c_int),
                ("pad", c_int)]


EXPORTS.update({
    "gm_maxpool2d_fwd_bf16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gm_bn_relu_maxpool2d_fwd_bf16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gm_bn_relu_maxpool2d_fwd_grouped_bf16": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                                      c_void_p, c_void_p]),
    "gm_bn_relu_maxpool2d_bwd_grouped_bf16": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                                      c_void_p, c_size_t, c_void_p]),
    "gm_bn_relu_maxpool2d_bwd_stats_grouped_bf16": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                                            c_void_p, c_void_p, c_size_t, c_void_p, c_void_p,
                                                            c_void_p]),
    "gm_conv_stem_stats_rows": (c_int, [c_void_p, c_int]),
    "gm_conv2d_fwd_grouped_stats_bf16": (c_int, [c_void_p, c_int, c_void_p, c_void_p, ctypes.c_longlong, c_void_p,
                                                 c_void_p, c_int, c_void_p]),
    "gm_bn_fwd_stats_finalize_grouped": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p]),
    "gm_conv2d_fwd_bn_stats_floats": (c_size_t, [c_void_p, c_int]),
    "gm_conv2d_fwd_grouped_bn_stats_bf16": (c_int, [c_void_p, c_int, c_void_p, c_void_p, ctypes.c_longlong, c_void_p,
                                                    c_void_p, c_size_t, c_void_p, c_void_p, c_size_t, c_void_p]),
    "gm_bn_fwd_apply_grouped_bf16": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p]),
    "gm_conv2d_dgrad_bn_stats_floats": (c_size_t, [c_void_p, c_int]),
    "gm_conv2d_dgrad_grouped_bn_stats_bf16": (c_int, [c_void_p, c_int, c_void_p, c_void_p, ctypes.c_longlong,
                                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                                      c_void_p, c_void_p, c_size_t, c_void_p]),
    "gm_bn_bwd_stats_coef_offset": (c_size_t, [c_int, c_int, c_int]),
    "gm_bn_bwd_stats_finalize_grouped": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p]),
    "gm_bn_bwd_apply_grouped_bf16": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p]),
    "gm_maxpool2d_bwd_bf16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
})


class ConvF32(ctypes.Structure):
    _fields_ = [("mode", c_int), ("d", ConvDesc), ("x", c_void_p), ("w", c_void_p), ("dy", c_void_p),
                ("out", c_void_p), ("addend", c_void_p), ("accumulate", c_int), ("pad0", c_int)]


GM_CONV_FWD, GM_CONV_DGRAD, GM_CONV_WGRAD = 0, 1, 2

EXPORTS.update({
    "gm_conv2d_f32_scratch": (c_size_t, [c_void_p]),
    "gm_conv2d_f32": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "gm_bn_fwd_train_f32": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "gm_bn_fwd_infer_f32": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "gm_bn_bwd_f32": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "gm_maxpool2d_fwd_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gm_maxpool2d_bwd_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
})

GM_FAULT_BN_SPIN, GM_FAULT_SPLITK_SPIN = 1, 2

EXPORTS.update({
    "gm_device_faults": (c_int, [ctypes.POINTER(ctypes.c_uint), c_int]),
    "gm_set_spin_limit": (c_int, [ctypes.c_uint]),
    "gm_bn_set_concurrency": (c_int, [c_int]),
    "gm_bn_set_fused_mode": (c_int, [c_int]),
    "gm_set_residency": (c_int, [c_int, c_int, c_int]),
    "gm_get_residency": (c_int, [ctypes.POINTER(c_int), ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
})


def set_residency(streams=None, sharers=None, reserved_cus=None):
    """Update the library's device residency plan (gm_set_residency); None keeps a field."""
    cur = get_residency()
    new = (cur[0] if streams is None else int(streams), cur[1] if sharers is None else int(sharers),
           cur[2] if reserved_cus is None else int(reserved_cus))
    check(load().gm_set_residency(*new), "gm_set_residency")
    return new


def get_residency():
    a, b, c = c_int(0), c_int(0), c_int(0)
    check(load().gm_get_residency(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), "gm_get_residency")
    return a.value, b.value, c.value


_fault_reset_hooks = []


def on_fault_reset(fn):
    """Register fn() to run when check_device_faults() finds a fault (state repair)."""
    _fault_reset_hooks.append(fn)
    return fn


def device_faults(clear=False):
    """OR of the library's sticky device fault words (synchronises the device)."""
    v = ctypes.c_uint(0)
    check(load().gm_device_faults(ctypes.byref(v), int(clear)), "gm_device_faults")
    return v.value


def check_device_faults(clear=True):
    """Raise if an in-launch hand-off (fused BatchNorm, split-K turnstile) timed out
    since the last check: its outputs were poisoned with NaN instead of stale data."""
    v = device_faults(clear)
    if v:
        for hook in _fault_reset_hooks:  # e.g. re-zero split-K turnstile words left mid-hand-off
            hook()
        what = [n for b, n in ((GM_FAULT_BN_SPIN, "fused BatchNorm coefficient hand-off"),
                               (GM_FAULT_SPLITK_SPIN, "split-K convolution turnstile")) if v & b]
        raise GreedyMMLError(f"device fault 0x{v:x}: {', '.join(what) or 'unknown'} timed out "
                             "(grid not co-resident?); the affected outputs are NaN")


class ViewsNorm(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("flip", c_void_p), ("B", c_int), ("V", c_int), ("H", c_int), ("W", c_int),
                ("C", c_int), ("mean", c_float * 4), ("std", c_float * 4), ("out", c_void_p), ("dtype", c_int),
                ("layout", c_int)]


EXPORTS.update({
    "gm_views_normalize": (c_int, [c_void_p, c_void_p]),
})

EXPORTS.update({
    "gm_conv_set_pipe": (c_int, [c_int]),
    "gm_conv_set_halo": (c_int, [c_int]),
    "gm_conv_set_h9": (c_int, [c_int]),
    "gm_conv_set_wgrad_staging": (c_int, [c_int]),
    "gm_conv_set_splitk": (c_int, [c_int]),
    "gm_conv_set_wgrad_loop": (c_int, [c_int]),
    "gm_conv_set_1x1_gemm": (c_int, [c_int]),
    "gm_conv_set_rw": (c_int, [c_int]),
    "gm_conv_set_stem": (c_int, [c_int]),
    "gm_conv_set_wgrad_stem": (c_int, [c_int]),
})
