"""Channels-last strided / broadcast copies (csrc/strided.hip): bit-identical to the torch ops they
replace -- the strided pick x[:, :, ::s, ::s] of the downsample's backward, the add of its input
gradient at the strided positions (torch's bf16 add_: fp32 sum, one rounding), and the average
pool's gradient broadcast over H x W. Odd sizes, strides 1-3, channels 8-512; rejects."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(2, 64, 56, 56, 2), (3, 256, 13, 13, 2), (1, 8, 7, 9, 3), (2, 512, 14, 14, 2), (4, 16, 5, 6, 1)]


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("N,C,H,W,s", SHAPES)
def test_strided_pick_and_add_match_torch(dev, N, C, H, W, s):
    from distributedauc_amd import ops

    g = torch.Generator(device=dev).manual_seed(N * 7 + C + H)
    x = _cl(torch.randn((N, C, H, W), device=dev, generator=g).to(torch.bfloat16))
    got = ops.strided_pick(x, s)
    ref = x[:, :, ::s, ::s]
    assert got.is_contiguous(memory_format=torch.channels_last) and got.shape == ref.shape
    assert torch.equal(got, ref)
    src = _cl(torch.randn(ref.shape, device=dev, generator=g).to(torch.bfloat16))
    a, b = x.clone(memory_format=torch.channels_last), x.clone(memory_format=torch.channels_last)
    ops.strided_add_(a, src, s)
    b[:, :, ::s, ::s].add_(src)
    assert torch.equal(a.view(torch.int16), b.view(torch.int16))


@pytest.mark.parametrize("N,C,H,W", [(256, 2048, 7, 7), (3, 8, 1, 1), (2, 64, 5, 3)])
def test_broadcast_hw_matches_expand(dev, N, C, H, W):
    from distributedauc_amd import ops

    gs = torch.randn((N, C, 1, 1), device=dev).to(torch.bfloat16)
    got = ops.broadcast_hw(gs, H, W)
    assert got.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(got, gs.expand(N, C, H, W))


def test_strided_rejects(dev):
    from distributedauc_amd import ops

    x = _cl(torch.zeros((1, 12, 4, 4), device=dev, dtype=torch.bfloat16))
    with pytest.raises(ValueError):
        ops.strided_pick(x, 2)  # C % 8
    y = torch.zeros((1, 16, 4, 4), device=dev, dtype=torch.bfloat16)  # NCHW
    with pytest.raises(ValueError):
        ops.strided_pick(y, 2)
    z = _cl(torch.zeros((1, 16, 4, 4), device=dev, dtype=torch.bfloat16))
    with pytest.raises(ValueError):
        ops.strided_add_(z, _cl(torch.zeros((1, 16, 3, 2), device=dev, dtype=torch.bfloat16)), 2)
