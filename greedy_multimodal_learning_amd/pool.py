"""Stem MaxPool2d on the HIP kernels (NHWC bf16, 1-byte argmax).

`GMMaxPool2d` is an `nn.MaxPool2d`; bf16 channels_last CUDA inputs (C % 8 == 0,
dilation 1, floor mode, no return_indices) run `gm_maxpool2d_fwd_bf16` /
`gm_maxpool2d_bwd_bf16`, everything else PyTorch's max_pool2d.  Reference:
torchvision ResNet `maxpool` as called at src/model.py:65-106.
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
        L.check(lib.gm_maxpool2d_fwd_bf16(ctypes.byref(d), x.data_ptr(), y.data_ptr(), idx.data_ptr(),
                                          L.stream_of(x.device)), "gm_maxpool2d_fwd_bf16")
        ctx.save_for_backward(idx)
        ctx.meta = (N, C, H, W, k, s, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = L.load()
        (idx,) = ctx.saved_tensors
        N, C, H, W, k, s, pad = ctx.meta
        dy = dy.to(torch.bfloat16)
        dy = dy if dy.is_contiguous(memory_format=CL) else dy.contiguous(memory_format=CL)
        dx = torch.empty(N, C, H, W, device=dy.device, dtype=torch.bfloat16, memory_format=CL)
        d = L.PoolDesc(N, H, W, C, k, s, pad)
        L.check(lib.gm_maxpool2d_bwd_bf16(ctypes.byref(d), dy.data_ptr(), idx.data_ptr(), dx.data_ptr(),
                                          L.stream_of(dy.device)), "gm_maxpool2d_bwd_bf16")
        return dx, None, None, None


class GMMaxPool2d(nn.MaxPool2d):
    def forward(self, x):
        k, s, p, dil = _pair1(self.kernel_size), _pair1(self.stride), _pair1(self.padding), _pair1(self.dilation)
        if (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0
                and None not in (k, s, p) and dil == 1 and not self.ceil_mode and not self.return_indices
                and k <= 15 and 2 * p <= k):
            return _PoolFn.apply(x, k, s, p)
        return super().forward(x)
