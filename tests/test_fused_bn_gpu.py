"""Fused BatchNorm + add + ReLU (csrc/bn_act.hip) against torch's own ops on the same inputs.

Reference: F.batch_norm(training=True) -> + residual -> relu, evaluated in fp64 (CPU) from the
same (bf16-rounded, for the bf16 path) inputs; autograd of that expression for the grads.
Tolerances: fp32 path 2e-5 relative to the tensor's scale (one-pass shifted statistics vs
torch's Welford); bf16 path: outputs are bf16, so |got - ref| <= 1/128 of the scale plus
one bf16 ulp of the value (the reference is rounded once more by the cast).
Running statistics: 1e-5 relative (fp32 path) / 1e-3 (bf16 inputs, same statistics).
"""
from __future__ import annotations

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref(x, bn, relu, res):
    """torch reference in fp64 on the CPU from the same inputs (copies of bn's buffers are updated).
    (fp64: torch's GPU fp32 batch_norm itself loses digits to E[x^2] - E[x]^2 on tiny M.)"""
    xr = x.detach().cpu().double().requires_grad_(True)
    w = bn.weight.detach().cpu().double().requires_grad_(True)
    b = bn.bias.detach().cpu().double().requires_grad_(True)
    rr = res.detach().cpu().double().requires_grad_(True) if res is not None else None
    rm, rv = bn.running_mean.cpu().double(), bn.running_var.cpu().double()
    y = F.batch_norm(xr, rm, rv, w, b, training=True, momentum=bn.momentum, eps=bn.eps)
    if rr is not None:
        y = y + rr
    if relu:
        y = F.relu(y)
    return y, xr, w, b, rr, rm, rv


def _close(got, ref, tol, scale=None):
    bf16 = got.dtype == torch.bfloat16
    got, ref = got.detach().cpu().double(), ref.detach().cpu().double()
    scale = ref.abs().max().clamp_min(1e-12) if scale is None else max(float(scale), float(ref.abs().max()))
    err = (got - ref).abs()
    ok = err <= tol * scale + ref.abs() * (2 ** -8 if bf16 else 0)
    return bool(ok.all()), float(err.max() / scale)


SHAPES = [(4, 64, 7, 9), (2, 256, 5, 5), (3, 2048, 3, 3), (8, 128, 14, 14), (2, 64, 1, 1), (2, 32, 33, 17)]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("mode", ["relu", "res_relu", "plain"])
def test_bn_act_matches_torch(dev, dtype, shape, mode):
    from distributedauc_amd.fused_bn import bn_act, supported

    torch.manual_seed(hash((shape, mode)) & 0xFFFF)
    N, C, H, W = shape
    x = (torch.randn(shape, device=dev) * 1.7 + 0.3).to(dtype).contiguous(memory_format=torch.channels_last)
    res = (torch.randn(shape, device=dev).to(dtype).contiguous(memory_format=torch.channels_last)
           if mode == "res_relu" else None)
    relu = mode != "plain"
    bn = nn.BatchNorm2d(C).to(dev).train()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.1, 0.1)
        bn.running_var.uniform_(0.9, 1.1)
    assert supported(x)
    yref, xr, w, b, rr, rm, rv = _ref(x, bn, relu, res)
    xg = x.detach().clone().requires_grad_(True)
    rg = res.detach().clone().requires_grad_(True) if res is not None else None
    y = bn_act(xg, bn, relu, rg)
    assert y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    tol = 2e-5 if dtype == torch.float32 else 2 ** -7
    ok, e = _close(y, yref, tol)
    assert ok, ("forward", e)
    rs_tol = 1e-5 if dtype == torch.float32 else 1e-3
    assert torch.allclose(bn.running_mean.cpu().double(), rm, rtol=rs_tol, atol=rs_tol)
    assert torch.allclose(bn.running_var.cpu().double(), rv, rtol=rs_tol, atol=rs_tol)
    assert int(bn.num_batches_tracked) == 1

    dy = torch.randn(shape, device=dev).to(dtype).contiguous(memory_format=torch.channels_last)
    yref.backward(dy.cpu().double())
    y.backward(dy)
    # dx = gamma*invstd*(g - mean g - xhat mean(g xhat)) cancels when M is tiny: its error is
    # relative to the scale of the terms, gamma*invstd*|g|
    xd = x.detach().cpu().double()
    invstd = 1.0 / torch.sqrt(xd.var(dim=(0, 2, 3), unbiased=False) + bn.eps)
    term = float((w.detach().abs() * invstd).max() * dy.detach().cpu().double().abs().max())
    for got, ref, name in ((xg.grad, xr.grad, "dx"), (bn.weight.grad, w.grad, "dgamma"),
                           (bn.bias.grad, b.grad, "dbeta")):
        ok, e = _close(got, ref, tol if name == "dx" else 1e-4, term if name == "dx" else None)
        assert ok, (name, e)
    if rg is not None:
        ok, e = _close(rg.grad, rr.grad, 0)
        assert ok, ("dres", e)


def test_bn_act_deterministic(dev):
    from distributedauc_amd.fused_bn import bn_act

    x = torch.randn(16, 256, 28, 28, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = []
    for _ in range(2):
        bn = nn.BatchNorm2d(256).to(dev).train()
        xg = x.clone().requires_grad_(True)
        y = bn_act(xg, bn, True, None)
        y.backward(torch.ones_like(y))
        outs.append((y, xg.grad, bn.weight.grad, bn.running_var.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_bn_act_rejects_unsupported(dev):
    from distributedauc_amd.fused_bn import bn_act, supported

    bn = nn.BatchNorm2d(96).to(dev).train()
    x = torch.randn(2, 96, 4, 4, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert not supported(x)
    with pytest.raises(ValueError):
        bn_act(x, bn)
    bn64 = nn.BatchNorm2d(64).to(dev).train()
    x_nchw = torch.randn(2, 64, 4, 4, device=dev)
    assert not supported(x_nchw)
    with pytest.raises(ValueError):
        bn_act(x_nchw, bn64)


def test_resnet_fused_matches_unfused(dev):
    """A ResNet-50 training step (channels-last) three ways: fp32 torch (the reference), bf16
    autocast with torch's BN/add/relu, bf16 autocast with the fused kernels. Summed over 3 seeds
    (tests/bf16_step_compare.py), the fused run must be as close to the fp32 reference as torch's
    own bf16 run is: logits max error <= 2x torch's + 1e-3; every parameter gradient's L2 error
    <= 2x torch bf16's + 1e-3 of its norm; every BN running statistic's max error likewise."""
    from bf16_step_compare import compare

    compare(dev, fused_bn=True, gemm_1x1=False, check_buffers=True)


def test_resnet_fused_counts_batches_once(dev):
    """Fused training forwards bump every BN's num_batches_tracked once (one multi-tensor launch)."""
    from distributedauc_amd.backbone import resnet18

    net = resnet18().to(dev).to(memory_format=torch.channels_last).set_fused_bn(True).train()
    x = torch.randn(4, 3, 32, 32, device=dev).contiguous(memory_format=torch.channels_last)
    net(x)
    net(x)
    counts = {n: int(b) for n, b in net.named_buffers() if n.endswith("num_batches_tracked")}
    assert counts and set(counts.values()) == {2}, counts
    net.eval()
    net(x)
    assert {int(b) for n, b in net.named_buffers() if n.endswith("num_batches_tracked")} == {2}


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("residual", [False, True])
def test_bn_relu_mask_matches_y_path(dev, dtype, residual):
    """Round 5: the forward's 1-bit ReLU mask (one byte per 16-byte vector) is exactly `y > 0` on the
    stored y -- zeros, negative zeros, values whose bf16 rounding lands on a denormal or on zero,
    +inf and NaN included -- and the backward that reads it gives dx, dres, dgamma and dbeta bit for
    bit as the backward that reads y (the layout: element i of vector v is bit i of mask byte v)."""
    from distributedauc_amd import _lib
    from distributedauc_amd.fused_bn import _DTYPES
    from distributedauc_amd.ops import _ptr, _stream, check, workspaces

    g = torch.Generator(device=dev).manual_seed(21)
    N, C, H, W = 4, 64, 6, 5
    x = torch.randn(N, C, H, W, device=dev, generator=g).to(dtype).contiguous(memory_format=torch.channels_last)
    flat = x.permute(0, 2, 3, 1).reshape(-1)  # channels-last order
    flat[::97] = 0.0
    flat[5::211] = float("nan")
    flat[7::223] = float("inf")
    res = torch.randn(N, C, H, W, device=dev, generator=g).to(dtype).contiguous(memory_format=torch.channels_last)
    # shift/scale so that many outputs sit just above / below zero, some in the denormal range
    gamma = torch.full((C,), 1e-38, device=dev)
    gamma[: C // 2] = 1.0
    beta = torch.zeros(C, device=dev)
    M = N * H * W
    L = _lib.load()
    ws = workspaces.get(dev, "bn_mask_test", L.dauc_bn_workspace_size(M, C))
    y = torch.empty_like(x)
    mask = torch.full((M * C * x.element_size() // 16,), 0xAA, dtype=torch.uint8, device=dev)
    mean, invstd = torch.empty(C, device=dev), torch.empty(C, device=dev)
    rp = res if residual else None
    check(L.dauc_bn_act_forward(_ptr(x), _DTYPES[dtype], M, C, _ptr(rp), 1, _ptr(gamma), _ptr(beta), None, None,
                                0.1, 1e-5, _ptr(y), _ptr(mask), _ptr(mean), _ptr(invstd), _ptr(ws), ws.numel(),
                                _stream(dev)), "forward")
    yv = y.permute(0, 2, 3, 1).reshape(-1).float()
    vec = 16 // x.element_size()
    bits = (yv > 0).view(-1, vec).to(torch.int32)
    want = (bits << torch.arange(vec, device=dev, dtype=torch.int32)).sum(1).to(torch.uint8)
    assert torch.equal(mask, want)
    assert bool((yv > 0).any()) and bool((yv == 0).any())
    dy = torch.randn(N, C, H, W, device=dev, generator=g).to(dtype).contiguous(memory_format=torch.channels_last)
    outs = []
    for use_mask in (False, True):
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if residual else None
        dgamma, dbeta = torch.empty(C, device=dev), torch.empty(C, device=dev)
        check(L.dauc_bn_act_backward(_ptr(dy), None if use_mask else _ptr(y), _ptr(mask) if use_mask else None,
                                     _ptr(x), _DTYPES[dtype], M, C, 1, _ptr(gamma), _ptr(mean), _ptr(invstd),
                                     _ptr(dres), _ptr(dx), _ptr(dgamma), _ptr(dbeta), _ptr(ws), ws.numel(),
                                     _stream(dev)), "backward")
        outs.append([t.view(torch.int16 if t.dtype == torch.bfloat16 else torch.int32).clone()
                     for t in (dx, dgamma, dbeta) + ((dres,) if residual else ())])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
