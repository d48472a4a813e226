"""Stem MaxPool2d on the HIP kernels (NHWC bf16 or fp32, 1-byte argmax).

`GMMaxPool2d` is an `nn.MaxPool2d`; CUDA inputs (C % 8 == 0, dilation 1, floor
mode, no return_indices) run `gm_maxpool2d_{fwd,bwd}_{bf16,f32}` on channels_last
activations (bf16: the engine's trunk; fp32: the reference's own arithmetic).
There is no PyTorch max_pool2d path: CPU tensors and other configurations raise.
Reference: torchvision ResNet `maxpool` as called at src/model.py:65-106.
"""
import ctypes

import torch
import torch.nn as nn

from . import _lib as L

CL = torch.channels_last


def _pair1(v):
    if isinstance(v, (tuple, list)):
        if len(v) != 2 or v[0] != v[1]:
            return None
        return int(v[0])
    return int(v)


class _PoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, pad):
        lib = L.load()
        x = x if x.is_contiguous(memory_format=CL) else x.contiguous(memory_format=CL)
        N, C, H, W = x.shape
        P, Q = (H + 2 * pad - k) // s + 1, (W + 2 * pad - k) // s + 1
        y = torch.empty(N, C, P, Q, device=x.device, dtype=x.dtype, memory_format=CL)
        idx = torch.empty(N, P, Q, C, device=x.device, dtype=torch.uint8)
        d = L.PoolDesc(N, H, W, C, k, s, pad)
        f32 = x.dtype == torch.float32
        fn = lib.gm_maxpool2d_fwd_f32 if f32 else lib.gm_maxpool2d_fwd_bf16
        L.check(fn(ctypes.byref(d), x.data_ptr(), y.data_ptr(), idx.data_ptr(), L.stream_of(x.device)),
                "gm_maxpool2d_fwd")
        ctx.save_for_backward(idx)
        ctx.meta = (N, C, H, W, k, s, pad, x.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = L.load()
        (idx,) = ctx.saved_tensors
        N, C, H, W, k, s, pad, dt = ctx.meta
        dy = dy.to(dt)
        dy = dy if dy.is_contiguous(memory_format=CL) else dy.contiguous(memory_format=CL)
        dx = torch.empty(N, C, H, W, device=dy.device, dtype=dt, memory_format=CL)
        d = L.PoolDesc(N, H, W, C, k, s, pad)
        fn = lib.gm_maxpool2d_bwd_f32 if dt == torch.float32 else lib.gm_maxpool2d_bwd_bf16
        L.check(fn(ctypes.byref(d), dy.data_ptr(), idx.data_ptr(), dx.data_ptr(), L.stream_of(dy.device)),
                "gm_maxpool2d_bwd")
        return dx, None, None, None


class GMMaxPool2d(nn.MaxPool2d):
    def forward(self, x):
        k, s, p, dil = _pair1(self.kernel_size), _pair1(self.stride), _pair1(self.padding), _pair1(self.dilation)
        if not x.is_cuda:
            raise L.GreedyMMLError("GMMaxPool2d: runs on libgreedymml_hip.so only (got a CPU tensor)")
        if not (x.dtype in (torch.bfloat16, torch.float32) and x.dim() == 4 and x.shape[1] % 8 == 0
                and None not in (k, s, p) and dil == 1 and not self.ceil_mode and not self.return_indices
                and k <= 15 and 2 * p <= k):
            raise L.GreedyMMLError("GMMaxPool2d: needs bf16/fp32 [N,C,H,W] with C % 8 == 0, square k <= 15, "
                                   "pad <= k/2, dilation 1, floor mode")
        return _PoolFn.apply(x, k, s, p)
