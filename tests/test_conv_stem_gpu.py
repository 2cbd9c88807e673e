"""The 7x7 / stride-2 / pad-3 stem convolution on csrc/conv_stem.hip (dauc_conv7x7s2_stem_*).

Reference: imagenet/resnet.py:145 (conv1) under main.py:311-326's forward / backward. Oracle: the
same convolution in fp64 on the CPU (torch.nn.functional.conv2d on the bf16 operands widened to
fp64). Tolerances: the forward is one bf16 rounding of an fp32 sum, so |y - ref| <= |ref| 2^-8 +
(fp32 accumulation, 1e-5 of the largest output); the weight gradient is an fp32 sum over every
output pixel (per-workgroup slabs summed in a fixed order, in two levels on the full grid), within
2e-5 of its largest entry.
Both are bitwise reproducible run to run.
"""
from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

# (7, 224, 64): 784 row tasks >= the 768-workgroup grid, so the weight gradient's two-level slab sum
SHAPES = [(2, 224, 224), (1, 17, 23), (3, 40, 300), (1, 1, 1), (5, 8, 9), (2, 2, 257), (7, 224, 64)]


def _inputs(dev, N, H, W, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn((N, 3, H, W), device=dev, generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn((64, 3, 7, 7), device=dev, generator=g) / 12).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    dy = torch.randn((N, 64, Ho, Wo), device=dev, generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    return x, w, dy


@pytest.mark.parametrize("N,H,W", SHAPES)
def test_stem_forward_matches_fp64(dev, N, H, W):
    from distributedauc_amd import ops

    x, w, _ = _inputs(dev, N, H, W, N * 100 + H + W)
    y = ops.stem_conv_forward(x, w)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    ref = F.conv2d(x.cpu().double(), w.cpu().double(), stride=2, padding=3)
    assert y.shape == ref.shape
    err = (y.cpu().double() - ref).abs()
    excess = float((err - ref.abs() * 2 ** -8).max())
    assert excess <= 1e-5 * float(ref.abs().max()), excess
    assert torch.equal(y, ops.stem_conv_forward(x, w))


@pytest.mark.parametrize("N,H,W", SHAPES)
def test_stem_wgrad_matches_fp64(dev, N, H, W):
    from distributedauc_amd import ops

    x, _, dy = _inputs(dev, N, H, W, N * 10 + H * 3 + W)
    dw = ops.stem_conv_wgrad(x, dy)
    assert dw.dtype == torch.float32 and dw.is_contiguous(memory_format=torch.channels_last)
    xd = x.cpu().double()
    wd = torch.zeros((64, 3, 7, 7), dtype=torch.float64, requires_grad=True)
    F.conv2d(xd, wd, stride=2, padding=3).backward(dy.cpu().double())
    ref = wd.grad
    scale = float(ref.abs().max())
    err = float((dw.cpu().double() - ref).abs().max())
    assert err <= 2e-5 * scale + 1e-30, (err, scale)
    assert torch.equal(dw, ops.stem_conv_wgrad(x, dy))  # fixed summation order


@pytest.mark.timeout(300)
def test_stem_resnet50_b256(dev):
    """The headline shape ([256, 3, 224, 224]) against torch's fp32 convolution on the GPU: forward
    within bf16 rounding, weight gradient within fp32 summation noise."""
    from distributedauc_amd import ops

    x, w, dy = _inputs(dev, 256, 224, 224, 3)
    y = ops.stem_conv_forward(x, w)
    with torch.autocast("cuda", enabled=False):
        ref = F.conv2d(x.float(), w.float(), stride=2, padding=3)
    err = (y.float() - ref).abs()
    assert float((err - ref.abs() * 2 ** -8).max()) <= 1e-4 * float(ref.abs().max())
    del y, ref, err
    dw = ops.stem_conv_wgrad(x, dy)
    wf = torch.zeros((64, 3, 7, 7), device=dev, requires_grad=True)
    tf32 = torch.backends.cudnn.allow_tf32
    torch.backends.cudnn.allow_tf32 = False
    try:
        with torch.autocast("cuda", enabled=False):
            F.conv2d(x.float(), wf, stride=2, padding=3).backward(dy.float())
    finally:
        torch.backends.cudnn.allow_tf32 = tf32
    scale = float(wf.grad.abs().max())
    assert float((dw - wf.grad).abs().max()) <= 1e-3 * scale


def test_stem_rejects_unsupported(dev):
    from distributedauc_amd import _lib, ops

    x, w, dy = _inputs(dev, 1, 16, 16, 0)
    with pytest.raises(ValueError):
        ops.stem_conv_forward(x.contiguous(), w)  # NCHW
    with pytest.raises(ValueError):
        ops.stem_conv_forward(x, w[:32])
    with pytest.raises(ValueError):
        ops.stem_conv_wgrad(x, dy[:, :, :-1])
    with pytest.raises(TypeError):
        ops.stem_conv_forward(x.float().contiguous(memory_format=torch.channels_last), w)
    L = _lib.load()
    # the C ABI checks the geometry itself: Ho must be (H - 1) / 2 + 1
    rc = L.dauc_conv7x7s2_stem_forward(ops._ptr(x), ops._ptr(w), _lib.DTYPE_BF16, 1, 16, 16, 9, 8, ops._ptr(dy),
                                       ops._stream(dev))
    assert rc == _lib.DAUC_EINVAL
    assert ops.stem_conv_supported(x, w, 2, 3, 1, 1)
    assert not ops.stem_conv_supported(x, w, 1, 3, 1, 1)
    assert not ops.stem_conv_supported(x.contiguous(), w, 2, 3, 1, 1)
    assert not ops.stem_conv_supported(x, w.contiguous(), 2, 3, 1, 1)  # NCHW weight
    assert not ops.stem_conv_supported(x, w.float().contiguous(memory_format=torch.channels_last), 2, 3, 1, 1)


@pytest.mark.parametrize("col", [4, 12, 13, 31])
@pytest.mark.parametrize("val", [float("inf"), float("-inf"), float("nan")])
def test_stem_forward_nonfinite_neighbour(dev, col, val):
    """the forward pads each row's 21 window elements to 24 with zero weights; the
    three padded lanes hold the input column just right of the window (2 ow + 4). A non-finite
    value there must not reach that output (0 x Inf = NaN), as in torch's convolution: the set of
    non-finite outputs equals the fp64 reference's, and the finite ones match it as in
    test_stem_forward_matches_fp64. Every channel of the column and the image's last column."""
    from distributedauc_amd import ops

    x, w, _ = _inputs(dev, 2, 32, 32, 17 + col)
    for ch in range(3):
        x[1, ch, 5 + 7 * ch, col] = val
    y = ops.stem_conv_forward(x, w)
    ref = F.conv2d(x.cpu().double(), w.cpu().double(), stride=2, padding=3)
    yc = y.cpu().double()
    assert torch.equal(torch.isfinite(yc), torch.isfinite(ref))
    assert int((~torch.isfinite(ref)).sum()) > 0
    fin = torch.isfinite(ref)
    err = (yc[fin] - ref[fin]).abs()
    assert float((err - ref[fin].abs() * 2 ** -8).max()) <= 1e-5 * float(ref[fin].abs().max())
