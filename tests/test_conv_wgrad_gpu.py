"""The 3x3 convolution weight gradient kernel (csrc/conv_wgrad.hip, dauc_conv3x3_wgrad) against an
fp64 reference of the same bf16 operands.

Reference: the weight gradient autograd computes for the ResNet 3x3 convolutions (resnet.py:72-108,
main.py:326), here as torch's fp64 convolution backward on the CPU from the same bf16-rounded x and
dy. The kernel accumulates exact bf16 products in fp32 (MFMA), split over pixel chunks whose fp32
partials are summed in a fixed order: error within fp32 summation noise of the fp64 result
(<= 2e-5 of the tensor's scale here), and bitwise reproducible. Also the transposing LDS read's
lane map (tuning build probe) and the backbone path that uses the kernel.
"""
from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def test_transposing_read_lane_map(dev):
    """ds_read_b64_tr_b16 as the kernel uses it: lane l gets channel 16 + (l & 15) of pixel rows
    8 (l >> 4) .. 8 (l >> 4) + 7 -- the 16x16x32 MFMA operand fragment."""
    from distributedauc_amd import ops

    got = ops.probe_tr16().cpu()
    for lane in range(64):
        g, i = lane >> 4, lane & 15
        want = [(8 * g + j) * 64 + 16 + i for j in range(8)]
        assert got[lane].tolist() == want, (lane, got[lane].tolist(), want)


def _ref_wgrad(x, dy, stride):
    xr = x.detach().cpu().double()
    gr = dy.detach().cpu().double()
    Co, Ci = dy.shape[1], x.shape[1]
    w = torch.zeros((Co, Ci, 3, 3), dtype=torch.float64)
    return torch.ops.aten.convolution_backward(gr, xr, w, None, [stride] * 2, [1, 1], [1, 1], False, [0, 0], 1,
                                               [False, True, False])[1]


@pytest.mark.parametrize("form", ["auto", "gather", "window64", "window128", "shared64", "shared128"])
@pytest.mark.parametrize("N,Ci,Co,H,W,stride", [
    (2, 64, 64, 9, 11, 1), (3, 128, 64, 14, 14, 2), (1, 64, 192, 7, 5, 1), (4, 64, 128, 15, 13, 2),
    (2, 256, 256, 14, 14, 1), (5, 512, 512, 7, 7, 1), (1, 64, 64, 1, 1, 1), (2, 64, 64, 2, 3, 2),
    (3, 64, 64, 70, 9, 1), (2, 64, 128, 131, 5, 2), (1, 64, 64, 3, 70, 1), (2, 64, 64, 5, 131, 2)])
def test_conv3x3_wgrad_matches_fp64(dev, form, N, Ci, Co, H, W, stride):
    """Every form of the kernel: the window form (whole output rows per chunk, the taps read one
    staged input window) with 64- or 128-pixel chunks (Wo <= 64 / 128; the automatic choice takes
    128 where its rows fill 7/8 of the chunk), and the gather form (64-pixel chunks, one gathered
    tile per tap; wider images), and the window form with shared rows (stride 1: a chunk's output
    rows read its R + 2 input rows, per image Ho + 2, when R divides Ho or Ho divides R). The tuning
    build's dauc_set_wgrad_form(1 .. 5) forces one form (a window form that does not fit falls back
    to the gather form)."""
    from distributedauc_amd import _lib, ops

    if form == "auto":
        _check_wgrad(dev, N, Ci, Co, H, W, stride)
        return
    ops.set_wgrad_form({"gather": 1, "window64": 2, "window128": 3, "shared64": 4, "shared128": 5}[form])
    try:
        with _lib.using(_lib.tuning()):
            _check_wgrad(dev, N, Ci, Co, H, W, stride)
    finally:
        ops.set_wgrad_form(0)


def _check_wgrad(dev, N, Ci, Co, H, W, stride):
    from distributedauc_amd import ops

    g = torch.Generator(device=dev).manual_seed(N * 1000 + Ci + Co + H)
    x = torch.randn((N, Ci, H, W), device=dev, generator=g).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    dy = torch.randn((N, Co, Ho, Wo), device=dev, generator=g).to(torch.bfloat16)
    dy = dy.contiguous(memory_format=torch.channels_last)
    got = ops.conv3x3_wgrad(x, dy, stride)
    assert got.dtype == torch.float32 and got.is_contiguous(memory_format=torch.channels_last)
    ref = _ref_wgrad(x, dy, stride)
    scale = float(ref.abs().max())
    err = float((got.cpu().double() - ref).abs().max())
    assert err <= 2e-5 * scale, (err, scale)
    again = ops.conv3x3_wgrad(x, dy, stride)
    assert torch.equal(got, again)  # fixed summation order


@pytest.mark.timeout(300)
@pytest.mark.parametrize("C,H,stride", [(64, 56, 1), (128, 56, 2), (256, 28, 2), (512, 14, 2), (512, 7, 1)])
def test_conv3x3_wgrad_resnet50_b256(dev, C, H, stride):
    """The bench's shapes (ResNet-50 b256 224^2: layer1 conv2, layer2.0 conv2, layer4 conv2) against
    torch's fp32 convolution backward on the GPU (fp32 operands from the same bf16 values)."""
    from distributedauc_amd import ops

    g = torch.Generator(device=dev).manual_seed(C + H)
    N = 256
    x = torch.relu(torch.randn((N, C, H, H), device=dev, generator=g)).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    Ho = (H - 1) // stride + 1
    dy = (torch.randn((N, C, Ho, Ho), device=dev, generator=g) * 1e-3).to(torch.bfloat16)
    dy = dy.contiguous(memory_format=torch.channels_last)
    got = ops.conv3x3_wgrad(x, dy, stride)
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), torch.zeros((C, C, 3, 3), device=dev), None,
                                                  [stride] * 2, [1, 1], [1, 1], False, [0, 0], 1,
                                                  [False, True, False])[1]
    finally:
        torch.backends.cudnn.deterministic = det
    scale = float(ref.abs().max())
    err = float((got - ref).abs().max())
    assert err <= 2e-4 * scale, (err, scale)


def test_conv3x3_wgrad_rejects_unsupported(dev):
    from distributedauc_amd import _lib, ops

    x = torch.randn((2, 48, 8, 8), device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn((2, 64, 8, 8), device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert not ops.conv3x3_wgrad_supported(x, dy, 1, 1, 1, 1)
    with pytest.raises(_lib.DaucError):
        ops.conv3x3_wgrad(x, dy, 1)  # Ci = 48: not a multiple of 64
    x = torch.randn((2, 64, 8, 8), device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with pytest.raises(_lib.DaucError):
        ops.conv3x3_wgrad(x, dy, 2)  # dy's 8 x 8 is not the stride-2 output size
    with pytest.raises(ValueError):
        ops.conv3x3_wgrad(x.contiguous(), dy, 1)
