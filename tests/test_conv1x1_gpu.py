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
@pytest.mark.parametrize("engines", [("gemm", "gemm", "gemm32"), ("conv", "conv", "conv"), ("gemm", "conv", "gemm8")])
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
    logits and every gradient within 2x the error torch's own bf16 autocast step makes."""
    from distributedauc_amd.backbone import build_backbone

    torch.manual_seed(0)
    base = build_backbone("resnet50", num_classes=2)
    x = torch.randn(8, 3, 64, 64, device=dev).contiguous(memory_format=torch.channels_last)
    runs = {}
    for name, amp, fast in (("fp32", False, False), ("bf16", True, False), ("fast", True, True)):
        net = build_backbone("resnet50", num_classes=2)
        net.load_state_dict(base.state_dict())
        net = net.to(dev).to(memory_format=torch.channels_last).train()
        net.set_fused_bn(fast).set_gemm_conv1x1(fast)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out = net(x)
        out[:, 1].sum().backward()
        runs[name] = (out.detach().float(), {n: p.grad.detach().float().flatten() for n, p in net.named_parameters()})
    ref_out, ref_g = runs["fp32"]
    e_b = float((runs["bf16"][0] - ref_out).abs().max())
    e_f = float((runs["fast"][0] - ref_out).abs().max())
    assert e_f <= 2 * e_b + 1e-3, (e_f, e_b)
    worse = []
    for n, g in ref_g.items():
        eb = float((runs["bf16"][1][n] - g).norm())
        ef = float((runs["fast"][1][n] - g).norm())
        if ef > 2 * eb + 1e-3 * float(g.norm()) + 1e-12:
            worse.append((n, ef, eb))
    assert not worse, worse
