"""1x1 convolutions as GEMMs (conv1x1.py) against an fp64 CPU convolution of the same inputs.

Every engine is forced once per direction (the autotuner's candidates), so each path is checked,
not only the one the timing picked. bf16 operands with fp32 accumulation: outputs within 2^-7 of
the tensor's scale plus one bf16 ulp; the fp32 weight gradient within 1e-2 of its scale (bf16
inputs, K = M up to 25k summed in fp32 slabs).
"""
from __future__ import annotations

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _err(got, ref):
    got, ref = got.detach().cpu().double(), ref.detach().cpu().double()
    return float((got - ref).abs().max() / ref.abs().max().clamp_min(1e-12))


@pytest.mark.parametrize("shape", [(4, 64, 256, 14), (2, 256, 64, 28), (8, 512, 2048, 7), (3, 128, 96, 5)])
@pytest.mark.parametrize("engines", [("gemm", "gemm", "gemm32"), ("conv", "conv", "conv"), ("gemm", "conv", "gemm8"),
                                     ("conv", "fconv", "gemm8")])
def test_conv1x1_engines(dev, shape, engines):
    from distributedauc_amd import conv1x1 as C

    N, cin, cout, H = shape
    torch.manual_seed(cin + cout)
    conv = nn.Conv2d(cin, cout, 1, bias=False).to(dev).to(memory_format=torch.channels_last)
    x = torch.randn(N, cin, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    M = N * H * H
    C.plans.clear()
    for d, e in zip(("fwd", "dgrad", "wgrad"), engines):
        if e.startswith("gemm") and d == "wgrad" and M % int(e[4:]):
            e = "conv"
        C.plans[(M, cin, cout, torch.bfloat16, d)] = e
    xg = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = C.conv1x1(conv, xg)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    gy = torch.randn_like(y)
    y.backward(gy)
    xr = x.detach().cpu().double().requires_grad_(True)
    wr = conv.weight.detach().cpu().double().to(torch.bfloat16).double().requires_grad_(True)
    yr = F.conv2d(xr, wr)
    yr.backward(gy.cpu().double())
    assert _err(y, yr) <= 2 ** -7, ("y", _err(y, yr))
    assert _err(xg.grad, xr.grad) <= 2 ** -7, ("dx", _err(xg.grad, xr.grad))
    assert conv.weight.grad.dtype == torch.float32 and conv.weight.grad.shape == conv.weight.shape
    assert _err(conv.weight.grad, wr.grad) <= 1e-2, ("dw", _err(conv.weight.grad, wr.grad))
    C.plans.clear()


def test_conv1x1_falls_back_for_strided(dev):
    from distributedauc_amd.conv1x1 import conv1x1

    conv = nn.Conv2d(64, 128, 1, stride=2, bias=False).to(dev)
    x = torch.randn(2, 64, 8, 8, device=dev)
    assert torch.equal(conv1x1(conv, x), conv(x))


def test_resnet_gemm_conv1x1_trains(dev):
    """ResNet-50 step with fused BN + GEMM 1x1 convs (autotuned engines) vs the fp32 torch step:
    summed over 3 seeds (tests/bf16_step_compare.py), logits and every gradient within 2x the
    error torch's own bf16 autocast step makes."""
    from bf16_step_compare import compare

    compare(dev, fused_bn=True, gemm_1x1=True)


@pytest.mark.timeout(900)
def test_resnet_fast_paths_at_bench_shape(dev):
    """The shipped default backbone (fused BN+add+ReLU, GEMM 1x1 convs on the shipped engine plan)
    at the bench's own shape, ResNet-50 b256 224x224 (BASELINE configs[1]), vs the fp32 torch
    step: logits, every gradient and the BN running stats within 2x the error of torch's own
    bf16 autocast step (2 seeds)."""
    from bf16_step_compare import compare

    compare(dev, fused_bn=True, gemm_1x1=True, check_buffers=True, batch=256, size=224, seeds=(0, 1))


@pytest.mark.parametrize("down", [0, 1, 2])
@pytest.mark.parametrize("owned", [False, True])
@pytest.mark.parametrize("acc_engine", ["gemm", "conv", "fconv"])
def test_conv1x1_skip_fuses_branch_gradient(dev, down, owned, acc_engine):
    """(conv1(x), skip) in one node: dx = dgrad(conv1) + d(skip), the sum accumulated by the GEMM
    (beta = 1, in place) or by an add after MIOpen's dgrad (or the forward convolution with W^T);
    skip = identity (down 0) or a 1x1
    downsample of stride 1 (GEMM) / 2 (MIOpen forward, backward as GEMMs on x[:, :, ::2, ::2] with the
    input gradient added at the strided positions; an odd H once); vs fp64 autograd of the two branches.
    Also: the incoming skip gradient is left untouched unless the caller marked it as owned."""
    from distributedauc_amd import conv1x1 as C

    torch.manual_seed(7 + down + 2 * owned)
    N, cin, width, H = 4, 256, 64, (13 if down == 2 and acc_engine == "fconv" else 14)
    conv = nn.Conv2d(cin, width, 1, bias=False).to(dev).to(memory_format=torch.channels_last)
    dconv = (nn.Conv2d(cin, 4 * width, 1, stride=down, bias=False).to(dev).to(memory_format=torch.channels_last)
             if down else None)
    x = torch.randn(N, cin, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    M = N * H * H
    C.plans.clear()
    C.plans[(M, cin, width, torch.bfloat16, "dgrad_acc")] = acc_engine
    xg = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        h, skip = C.conv1x1_skip(conv, xg, dconv, skip_grad_owned=owned)
    assert h.dtype == skip.dtype == torch.bfloat16
    if not down:
        assert torch.equal(skip, x)
    gh = torch.randn_like(h)
    gs = torch.randn_like(skip).contiguous(memory_format=torch.channels_last)
    gs_copy = gs.clone()
    torch.autograd.backward([h, skip], [gh, gs])
    if not owned:
        assert torch.equal(gs, gs_copy), "a gradient the node does not own was modified"
    xr = x.detach().cpu().double().requires_grad_(True)
    wr = conv.weight.detach().cpu().double().to(torch.bfloat16).double().requires_grad_(True)
    hr = F.conv2d(xr, wr)
    if down:
        wdr = dconv.weight.detach().cpu().double().to(torch.bfloat16).double().requires_grad_(True)
        sr = F.conv2d(xr, wdr, stride=down)
    else:
        sr = xr
    torch.autograd.backward([hr, sr], [gh.cpu().double(), gs_copy.cpu().double()])
    assert _err(h, hr) <= 2 ** -7 and _err(skip, sr) <= 2 ** -7
    assert _err(xg.grad, xr.grad) <= 2 ** -7, ("dx", _err(xg.grad, xr.grad))
    assert _err(conv.weight.grad, wr.grad) <= 1e-2, ("dw1", _err(conv.weight.grad, wr.grad))
    if down:
        assert _err(dconv.weight.grad, wdr.grad) <= 1e-2, ("dwd", _err(dconv.weight.grad, wdr.grad))
    C.plans.clear()


@pytest.mark.parametrize("S,n", [(1, 4), (8, 64 * 256), (32, 2048 * 512), (13, 1028), (128, 256 * 64)])
def test_slab_sum_matches_sequential_fp32(dev, S, n):
    """dauc_slab_sum: out = sum of S slabs in ascending slab order, bit-identical to sequential
    fp32 adds (the split-K weight-gradient reduction of the 1x1 convolutions)."""
    from distributedauc_amd import _lib
    from distributedauc_amd.ops import _ptr, _stream, check

    g = torch.Generator(device=dev).manual_seed(S * 7 + n)
    part = torch.randn((S, n), device=dev, generator=g) * torch.rand((S, 1), device=dev, generator=g) * 100
    out = torch.empty(n, device=dev)
    check(_lib.load().dauc_slab_sum(_ptr(part), S, n, _ptr(out), _stream(dev)), "dauc_slab_sum")
    ref = torch.zeros(n, device=dev)
    for s in range(S):
        ref += part[s]
    assert torch.equal(out, ref)
    assert _lib.load().dauc_slab_sum(_ptr(part), S, n - 2, _ptr(out), _stream(dev)) == _lib.DAUC_EINVAL
