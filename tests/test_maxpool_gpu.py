"""Stem max-pool kernels (csrc/maxpool.hip, pool.py) against torch's own GPU max-pool.

Reference: ``F.max_pool2d`` on the same channels-last CUDA tensor (torch's max_pool_forward_nhwc /
max_pool_backward_nhwc, the kernels the backbone ran before, resnet.py:205). Bar: bit-identical
outputs and input gradients (compared as raw bits, so NaN payloads and -0.0 count), including
ties, NaN, all -inf windows (torch's index-0 quirk) and windows clipped by the padding.
"""
from __future__ import annotations

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _bits(t: torch.Tensor) -> torch.Tensor:
    t = t.detach().contiguous(memory_format=torch.channels_last) if t.dim() == 4 else t.detach()
    return t.view(torch.int16 if t.element_size() == 2 else torch.int32).cpu()


def _run(x, dy, k, s, p, ours: bool):
    xi = x.detach().clone(memory_format=torch.channels_last).requires_grad_(True)
    if ours:
        from distributedauc_amd.pool import max_pool2d

        y = max_pool2d(xi, nn.MaxPool2d(k, s, p))
    else:
        y = F.max_pool2d(xi, k, s, p)
    y.backward(dy)
    return y, xi.grad


def _check(x, k, s, p, seed=0):
    g = torch.Generator(device=x.device).manual_seed(seed)
    N, C, H, W = x.shape
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = torch.randn((N, C, Ho, Wo), device=x.device, generator=g).to(x.dtype)
    dy = dy.contiguous(memory_format=torch.channels_last)
    y0, g0 = _run(x, dy, k, s, p, ours=False)
    y1, g1 = _run(x, dy, k, s, p, ours=True)
    assert y1.shape == y0.shape and y1.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(_bits(y1), _bits(y0)), "forward differs from torch"
    assert torch.equal(_bits(g1), _bits(g0)), "input gradient differs from torch"


WINDOWS = [(3, 2, 1), (2, 2, 0), (3, 1, 1), (5, 2, 2), (3, 3, 0), (1, 1, 0)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(2, 64, 28, 28), (3, 8, 7, 9), (1, 16, 1, 1), (2, 64, 13, 11), (1, 24, 2, 3)])
@pytest.mark.parametrize("win", WINDOWS)
def test_maxpool_matches_torch(dev, dtype, shape, win):
    k, s, p = win
    N, C, H, W = shape
    if (H + 2 * p - k) // s + 1 < 1 or (W + 2 * p - k) // s + 1 < 1:
        pytest.skip("window larger than the padded input")
    g = torch.Generator(device=dev).manual_seed(hash((shape, win)) & 0xFFFF)
    x = torch.randn(shape, device=dev, generator=g).to(dtype).contiguous(memory_format=torch.channels_last)
    _check(x, k, s, p)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_maxpool_ties_and_relu_zeros(dev, dtype):
    """Post-ReLU stem activations: many exact zeros and few levels -> ties in most windows."""
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.relu(torch.floor(torch.randn((4, 64, 30, 30), device=dev, generator=g) * 2) / 2)
    _check(x.to(dtype).contiguous(memory_format=torch.channels_last), 3, 2, 1)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_maxpool_nan_inf_and_signed_zero(dev, dtype):
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn((2, 16, 11, 12), device=dev, generator=g)
    m = torch.rand(x.shape, device=dev, generator=g)
    x = torch.where(m < 0.05, torch.full_like(x, float("nan")), x)
    x = torch.where((m > 0.05) & (m < 0.1), torch.full_like(x, float("inf")), x)
    x = torch.where((m > 0.1) & (m < 0.2), torch.full_like(x, float("-inf")), x)
    x = torch.where((m > 0.2) & (m < 0.3), torch.full_like(x, -0.0), x)
    x = torch.where((m > 0.3) & (m < 0.4), torch.zeros_like(x), x)
    _check(x.to(dtype).contiguous(memory_format=torch.channels_last), 3, 2, 1)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_maxpool_all_minus_inf(dev, dtype):
    """No element compares greater than -inf: torch records index 0 (the image's first pixel), so
    only windows covering pixel (0, 0) pass their gradient on, and only to it."""
    x = torch.full((2, 8, 9, 9), float("-inf"), device=dev)
    x[1, :, 4:, 4:] = 1.0
    _check(x.to(dtype).contiguous(memory_format=torch.channels_last), 3, 2, 1)
    _check(x.to(dtype).contiguous(memory_format=torch.channels_last), 3, 1, 1)


def test_maxpool_resnet50_stem_size(dev):
    """The bench's stem: [256, 64, 112, 112] bf16 -> [256, 64, 56, 56] (3, 2, 1)."""
    g = torch.Generator(device=dev).manual_seed(11)
    x = torch.relu(torch.randn((256, 64, 112, 112), device=dev, generator=g)).to(torch.bfloat16)
    _check(x.contiguous(memory_format=torch.channels_last), 3, 2, 1)


def test_maxpool_refuses_unsupported(dev):
    from distributedauc_amd.pool import max_pool2d, supported

    x = torch.randn((2, 12, 8, 8), device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert not supported(x)  # 12 channels: not a whole 16-byte vector of bf16
    with pytest.raises(ValueError):
        max_pool2d(x, nn.MaxPool2d(3, 2, 1))
    with pytest.raises(ValueError):
        max_pool2d(torch.randn((2, 16, 8, 8), device=dev).contiguous(memory_format=torch.channels_last),
                   nn.MaxPool2d(3, 2, 1, ceil_mode=True))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(256, 2048, 7, 7), (3, 16, 5, 4), (2, 8, 1, 1)])
def test_global_avgpool_channels_last_grad_matches_torch(dev, dtype, shape):
    """backbone._GlobalAvgPoolCL (the head's average pool, resnet.py:210): the same output and the
    same input-gradient bits as torch's AdaptiveAvgPool2d(1), the gradient channels-last."""
    from distributedauc_amd.backbone import _GlobalAvgPoolCL

    g = torch.Generator(device=dev).manual_seed(21)
    x = torch.randn(shape, device=dev, generator=g).to(dtype).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(shape[:2], device=dev, generator=g).to(dtype)
    xa = x.clone(memory_format=torch.channels_last).requires_grad_(True)
    ya = torch.flatten(nn.AdaptiveAvgPool2d(1)(xa), 1)
    ya.backward(dy)
    xb = x.clone(memory_format=torch.channels_last).requires_grad_(True)
    yb = torch.flatten(_GlobalAvgPoolCL.apply(xb), 1)
    yb.backward(dy)
    assert torch.equal(_bits(yb), _bits(ya))
    assert xb.grad.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(_bits(xb.grad), _bits(xa.grad))
