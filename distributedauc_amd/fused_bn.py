"""Fused BatchNorm + residual add + ReLU for the channels-last ResNet backbone (training mode).

The reference's blocks (resnet.py:47-64, 87-108, stem 203-206) run bn, the residual add and
relu as separate passes; under torch each is its own HBM round trip (MIOpen's three BN
kernels forward, three backward, plus the elementwise add and relu both ways). Here one
autograd node per BN layer calls ``dauc_bn_act_forward`` / ``dauc_bn_act_backward``
(csrc/bn_act.hip): two passes over the activation forward, two backward. With ReLU the forward
also writes a 1-bit-per-element mask of y > 0 and the backward reads it instead of y (both
backward passes are HBM-bound: 2 B less per element and pass in bf16).

Semantics are torch's ``F.batch_norm(training=True)`` followed by ``+ residual`` and
``relu``: batch mean and biased variance for the normalisation, running statistics
updated with the unbiased variance and ``momentum`` (or the cumulative average when
``momentum is None``), ``num_batches_tracked`` incremented. There is no CPU path: the
backbone falls back to torch's own modules only in eval mode (running statistics).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib
from .ops import _ptr, _stream, check, workspaces

__all__ = ["supported", "bn_act", "BnActFunction"]

_DTYPES = {torch.float32: 1, torch.bfloat16: 2}  # DAUC_DTYPE_F32 / DAUC_DTYPE_BF16


def supported(x: torch.Tensor) -> bool:
    """True if ``x`` [N, C, H, W] is a channels-last bf16/fp32 CUDA tensor the kernels take:
    C a multiple of the 16-byte vector with a power-of-two vector count (or a multiple of 256
    vectors), 16-byte aligned."""
    if x.dim() != 4 or x.device.type != "cuda" or x.dtype not in _DTYPES:
        return False
    if not x.is_contiguous(memory_format=torch.channels_last) or x.data_ptr() % 16:
        return False
    vec = 16 // x.element_size()
    C = x.shape[1]
    if C % vec:
        return False
    cv = C // vec
    tpr = min(cv, 256)
    return 256 % tpr == 0 and cv % tpr == 0


class BnActFunction(torch.autograd.Function):
    """y = relu?(batch_norm(x) + residual?) with the fused kernels; grads for x, gamma, beta, residual."""

    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, momentum, eps, relu):
        N, C, H, W = x.shape
        M = N * H * W
        dev = x.device
        L = _lib.load()
        y = torch.empty_like(x, memory_format=torch.channels_last)
        # the ReLU mask: one byte per 16-byte vector of y
        mask = torch.empty(M * C * x.element_size() // 16, dtype=torch.uint8, device=dev) if relu else None
        mean = torch.empty(C, dtype=torch.float32, device=dev)
        invstd = torch.empty(C, dtype=torch.float32, device=dev)
        ws = workspaces.get(dev, "bn", L.dauc_bn_workspace_size(M, C))
        if residual is not None:
            if residual.shape != x.shape or residual.dtype != x.dtype:
                raise ValueError("residual must match x in shape and dtype")
            residual = residual.contiguous(memory_format=torch.channels_last)
        check(L.dauc_bn_act_forward(_ptr(x), _DTYPES[x.dtype], M, C, _ptr(residual), int(relu), _ptr(weight),
                                    _ptr(bias), _ptr(running_mean), _ptr(running_var), float(momentum), float(eps),
                                    _ptr(y), _ptr(mask), _ptr(mean), _ptr(invstd), _ptr(ws), ws.numel(), _stream(dev)),
              "dauc_bn_act_forward")
        ctx.save_for_backward(x, mask, weight, mean, invstd)
        ctx.relu = bool(relu)
        ctx.has_residual = residual is not None
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, weight, mean, invstd = ctx.saved_tensors
        N, C, H, W = x.shape
        M = N * H * W
        dev = x.device
        L = _lib.load()
        dy = dy.contiguous(memory_format=torch.channels_last)
        if dy.dtype != x.dtype:
            dy = dy.to(x.dtype)
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        dres = torch.empty_like(x, memory_format=torch.channels_last) if ctx.has_residual else None
        dgamma = torch.empty(C, dtype=torch.float32, device=dev) if weight is not None else None
        dbeta = torch.empty(C, dtype=torch.float32, device=dev) if ctx.has_bias else None
        ws = workspaces.get(dev, "bn", L.dauc_bn_workspace_size(M, C))
        check(L.dauc_bn_act_backward(_ptr(dy), None, _ptr(mask), _ptr(x), _DTYPES[x.dtype], M, C, int(ctx.relu),
                                     _ptr(weight), _ptr(mean), _ptr(invstd), _ptr(dres), _ptr(dx), _ptr(dgamma),
                                     _ptr(dbeta), _ptr(ws), ws.numel(), _stream(dev)),
              "dauc_bn_act_backward")
        return dx, dgamma, dbeta, dres, None, None, None, None, None


def bn_act(x: torch.Tensor, bn: nn.BatchNorm2d, relu: bool = True,
           residual: torch.Tensor | None = None) -> torch.Tensor:
    """Training-mode ``relu?(bn(x) + residual?)`` through the fused kernels (x channels-last, on the GPU)."""
    if x.device.type != "cuda":
        raise RuntimeError("fused BN runs on the GPU only (libdauc.so); no CPU path")
    if not supported(x):
        raise ValueError(f"fused BN needs a channels-last bf16/fp32 tensor with a supported channel count, "
                         f"got {tuple(x.shape)} {x.dtype}")
    momentum = 0.0 if bn.momentum is None else bn.momentum
    rm, rv = (bn.running_mean, bn.running_var) if bn.track_running_stats else (None, None)
    if bn.track_running_stats and bn.num_batches_tracked is not None and not getattr(bn, "_dauc_counted", False):
        bn.num_batches_tracked.add_(1)
        if bn.momentum is None:  # cumulative moving average (torch semantics; syncs once)
            momentum = 1.0 / float(bn.num_batches_tracked.item())
    return BnActFunction.apply(x, bn.weight, bn.bias, residual, rm, rv, momentum, bn.eps, relu)
