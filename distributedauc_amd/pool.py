"""The backbone stem's max-pool (resnet.py:205, ``nn.MaxPool2d(3, 2, 1)``) through HIP kernels.

torch's NHWC max-pool saves an int64 index per output element; for the ResNet-50 b256 stem that is
411 MB written forward and read backward, more than the pooled activation itself, and its backward
kernel runs at a fraction of HBM bandwidth. ``dauc_maxpool2d_forward`` / ``_backward``
(csrc/maxpool.hip) save one int8 window position per element and reproduce torch's comparisons and
fp32 gradient summation order, so outputs and gradients are bit-identical to
``F.max_pool2d``. No CPU path: the backbone uses this node only on the GPU (``ResNet.set_fused_bn``).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib
from .ops import _ptr, _stream, check

__all__ = ["supported", "max_pool2d", "MaxPoolFunction"]

_DTYPES = {torch.float32: 1, torch.bfloat16: 2}  # DAUC_DTYPE_F32 / DAUC_DTYPE_BF16


def _out_size(n: int, k: int, s: int, p: int) -> int:
    return (n + 2 * p - k) // s + 1


def supported(x: torch.Tensor, kernel: int = 3, stride: int = 2, padding: int = 1) -> bool:
    """True if the kernels take ``x`` [N, C, H, W]: channels-last bf16/fp32 on the GPU, C a multiple of
    the 16-byte vector, 16-byte aligned, and a window torch accepts (pad <= kernel / 2)."""
    if x.dim() != 4 or x.device.type != "cuda" or x.dtype not in _DTYPES:
        return False
    if not x.is_contiguous(memory_format=torch.channels_last) or x.data_ptr() % 16:
        return False
    N, C, H, W = x.shape
    if N < 1 or C % (16 // x.element_size()) or kernel * kernel > 127 or 2 * padding > kernel:
        return False
    return _out_size(H, kernel, stride, padding) >= 1 and _out_size(W, kernel, stride, padding) >= 1


class MaxPoolFunction(torch.autograd.Function):
    """y = max_pool2d(x, kernel, stride, padding) (floor mode, dilation 1); int8 argmax saved."""

    @staticmethod
    def forward(ctx, x, kernel, stride, padding):
        N, C, H, W = x.shape
        Ho, Wo = _out_size(H, kernel, stride, padding), _out_size(W, kernel, stride, padding)
        y = torch.empty((N, C, Ho, Wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        idx = torch.empty((N, Ho, Wo, C), dtype=torch.int8, device=x.device)
        check(_lib.load().dauc_maxpool2d_forward(_ptr(x), _DTYPES[x.dtype], N, H, W, C, kernel, stride, padding,
                                                 _ptr(y), _ptr(idx), Ho, Wo, _stream(x.device)),
              "dauc_maxpool2d_forward")
        ctx.save_for_backward(idx)
        ctx.geom = (N, C, H, W, kernel, stride, padding, Ho, Wo)
        ctx.dtype = x.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        N, C, H, W, k, s, p, Ho, Wo = ctx.geom
        dy = dy.contiguous(memory_format=torch.channels_last)
        if dy.dtype != ctx.dtype:
            dy = dy.to(ctx.dtype)
        if dy.data_ptr() % 16:
            dy = dy.clone(memory_format=torch.channels_last)
        dx = torch.empty((N, C, H, W), dtype=ctx.dtype, device=dy.device, memory_format=torch.channels_last)
        check(_lib.load().dauc_maxpool2d_backward(_ptr(dy), _ptr(idx), _DTYPES[ctx.dtype], N, H, W, C, k, s, p,
                                                  Ho, Wo, _ptr(dx), _stream(dy.device)),
              "dauc_maxpool2d_backward")
        return dx, None, None, None


def _as_int(v) -> int:
    if isinstance(v, (tuple, list)):
        if len(set(v)) != 1:
            raise ValueError(f"square windows only, got {v}")
        v = v[0]
    return int(v)


def max_pool2d(x: torch.Tensor, pool: nn.MaxPool2d) -> torch.Tensor:
    """``pool(x)`` through the HIP kernels (x channels-last on the GPU); raises where they do not apply."""
    if x.device.type != "cuda":
        raise RuntimeError("the max-pool kernels run on the GPU only (libdauc.so); no CPU path")
    k, s, p = _as_int(pool.kernel_size), _as_int(pool.stride or pool.kernel_size), _as_int(pool.padding)
    if pool.ceil_mode or _as_int(pool.dilation) != 1 or pool.return_indices:
        raise ValueError("max-pool kernels: floor mode, dilation 1, no returned indices only")
    if not supported(x, k, s, p):
        raise ValueError(f"max-pool kernels need a channels-last bf16/fp32 tensor with C a multiple of the "
                         f"16-byte vector, got {tuple(x.shape)} {x.dtype}")
    return MaxPoolFunction.apply(x, k, s, p)
