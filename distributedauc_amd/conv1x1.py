"""Stride-1 1x1 convolutions of the channels-last backbone as plain GEMMs where that is faster.

In NHWC a 1x1 convolution is a GEMM over the [M, C] view of the activation (M = N*H*W):
    forward  y[M, Cout]     = x[M, Cin] @ W[Cout, Cin]^T
    dgrad    dx[M, Cin]     = dy[M, Cout] @ W
    wgrad    dW[Cout, Cin]  = dy^T @ x   (K = M: split over S slabs, fp32 partial sums)
MIOpen's implicit-GEMM convolutions zero their output before every launch and lose to hipBLASLt
on most ResNet-50 1x1 shapes (profiles/r01/probe_conv1x1.log), but not on all of them (the
large-M / small-C layer1 shapes favour MIOpen). So each (shape, direction) is timed once, on
first use, with both engines on the live stream (HIP events, best of 3) and the faster one is
kept - the cudnn.benchmark idea, per direction. Numerics: bf16 operands, fp32 accumulation,
bf16 activations / fp32 weight gradient (the fp32 master weight's grad is returned directly,
so autocast's cast-back kernel disappears too).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = ["conv1x1", "Conv1x1Function", "plans"]

plans: dict = {}  # (M, Cin, Cout, dtype, direction) -> engine


def _timed(fn, reps=3):
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    return best


_FORCE = os.environ.get("DAUC_CONV1X1", "auto")  # auto | gemm | conv (fixed engine: reproducible runs)


def _choose(key, candidates: dict):
    eng = plans.get(key)
    if eng is None and _FORCE != "auto":
        eng = next((n for n in candidates if n.startswith(_FORCE)), None)
        if eng == "gemm8" and "gemm32" in candidates:
            eng = "gemm32"
        if eng is not None:
            plans[key] = eng
    if eng is None:
        times = {name: _timed(fn) for name, fn in candidates.items()}
        eng = min(times, key=times.get)
        plans[key] = eng
    return eng


def _wgrad_gemm(g2, x2, slabs):
    M, cout = g2.shape
    cin = x2.shape[1]
    if slabs == 1:
        return torch.mm(g2.t(), x2, out_dtype=torch.float32)
    part = torch.bmm(g2.view(slabs, M // slabs, cout).transpose(1, 2), x2.view(slabs, M // slabs, cin),
                     out_dtype=torch.float32)
    return part.sum(0)


class Conv1x1Function(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight):
        N, cin, H, W = x.shape
        cout = weight.shape[0]
        M = N * H * W
        wc = weight.detach().reshape(cout, cin).to(x.dtype)
        x2 = x.permute(0, 2, 3, 1).reshape(M, cin)  # a view: x is channels-last contiguous
        with torch.autocast("cuda", enabled=False):
            key = (M, cin, cout, x.dtype, "fwd")
            eng = _choose(key, {"gemm": lambda: torch.mm(x2, wc.t()),
                                "conv": lambda: F.conv2d(x, wc.view(cout, cin, 1, 1))})
            if eng == "gemm":
                y = torch.mm(x2, wc.t()).view(N, H, W, cout).permute(0, 3, 1, 2)
            else:
                y = F.conv2d(x, wc.view(cout, cin, 1, 1)).contiguous(memory_format=torch.channels_last)
        ctx.save_for_backward(x, wc)
        ctx.wdtype = weight.dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        x, wc = ctx.saved_tensors
        N, cin, H, W = x.shape
        cout = wc.shape[0]
        M = N * H * W
        gy = gy.to(x.dtype).contiguous(memory_format=torch.channels_last)
        g2 = gy.permute(0, 2, 3, 1).reshape(M, cout)
        x2 = x.permute(0, 2, 3, 1).reshape(M, cin)
        w4 = wc.view(cout, cin, 1, 1)
        dx = dw = None
        with torch.autocast("cuda", enabled=False):
            if ctx.needs_input_grad[0]:
                key = (M, cin, cout, x.dtype, "dgrad")

                def conv_d():
                    return torch.ops.aten.convolution_backward(gy, x, w4, None, [1, 1], [0, 0], [1, 1], False,
                                                               [0, 0], 1, [True, False, False])[0]

                eng = _choose(key, {"gemm": lambda: torch.mm(g2, wc), "conv": conv_d})
                if eng == "gemm":
                    dx = torch.mm(g2, wc).view(N, H, W, cin).permute(0, 3, 1, 2)
                else:
                    dx = conv_d().contiguous(memory_format=torch.channels_last)
            if ctx.needs_input_grad[1]:
                key = (M, cin, cout, x.dtype, "wgrad")

                def conv_w():
                    return torch.ops.aten.convolution_backward(gy, x, w4, None, [1, 1], [0, 0], [1, 1], False,
                                                               [0, 0], 1, [False, True, False])[1]

                cands = {"conv": conv_w}
                for s in (8, 32, 128):
                    if M % s == 0 and M // s >= 64:
                        cands[f"gemm{s}"] = (lambda s=s: _wgrad_gemm(g2, x2, s))
                eng = _choose(key, cands)
                if eng == "conv":
                    dw = conv_w().reshape(cout, cin).to(ctx.wdtype)
                else:
                    dw = _wgrad_gemm(g2, x2, int(eng[4:])).to(ctx.wdtype)
                dw = dw.view(cout, cin, 1, 1)
        return dx, dw


def conv1x1(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """``conv(x)`` for a bias-free, stride-1, ungrouped 1x1 conv on a channels-last GPU tensor;
    anything else goes to the module itself."""
    if (conv.kernel_size != (1, 1) or conv.stride != (1, 1) or conv.groups != 1 or conv.bias is not None
            or conv.padding != (0, 0) or x.device.type != "cuda"
            or not x.is_contiguous(memory_format=torch.channels_last)):
        return conv(x)
    if torch.is_autocast_enabled("cuda") and x.dtype == torch.float32:
        x = x.to(torch.get_autocast_dtype("cuda"))
    return Conv1x1Function.apply(x, conv.weight)
