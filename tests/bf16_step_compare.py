"""Shared check for the backbone's bf16 fast paths: a ResNet-50 training step compared with the
fp32 torch step, against the error torch's own bf16 autocast step makes on the same inputs.

One step's bf16 error is noisy (the max |logit error| of one seed ranges 0.05-0.20 at logit scale
~0.8 for every bf16 variant, scripts/probe_conv_noise.py), so errors are summed over SEEDS seeds
before the comparison: sum(err_fast) <= 2 x sum(err_torch_bf16) + slack."""
from __future__ import annotations

import torch

SEEDS = (0, 1, 2)


def _step(dev, seed, amp: bool, fused_bn: bool, gemm_1x1: bool, batch: int = 8, size: int = 64):
    from distributedauc_amd.backbone import build_backbone

    torch.manual_seed(seed)
    net = build_backbone("resnet50", num_classes=2)
    x = torch.randn(batch, 3, size, size, device=dev).contiguous(memory_format=torch.channels_last)
    net = net.to(dev).to(memory_format=torch.channels_last).train()
    net.set_fused_bn(fused_bn)
    if gemm_1x1:
        net.set_gemm_conv1x1(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        out = net(x)
    out[:, 1].sum().backward()
    return (out.detach().float(), {n: p.grad.detach().float().flatten() for n, p in net.named_parameters()},
            {n: b.detach().float() for n, b in net.named_buffers()})


def compare(dev, fused_bn: bool, gemm_1x1: bool, check_buffers: bool = False, batch: int = 8, size: int = 64,
            seeds=SEEDS) -> None:
    e_out = [0.0, 0.0]
    e_grad: dict = {}
    g_norm: dict = {}
    e_buf: dict = {}
    b_max: dict = {}
    for seed in seeds:
        ref_out, ref_g, ref_b = _step(dev, seed, False, False, False, batch, size)
        tb = _step(dev, seed, True, False, False, batch, size)
        fa = _step(dev, seed, True, fused_bn, gemm_1x1, batch, size)
        e_out[0] += float((tb[0] - ref_out).abs().max())
        e_out[1] += float((fa[0] - ref_out).abs().max())
        for n, g in ref_g.items():
            eb, ef = e_grad.get(n, (0.0, 0.0))
            e_grad[n] = (eb + float((tb[1][n] - g).norm()), ef + float((fa[1][n] - g).norm()))
            g_norm[n] = g_norm.get(n, 0.0) + float(g.norm())
        for n, b in ref_b.items():
            eb, ef = e_buf.get(n, (0.0, 0.0))
            e_buf[n] = (eb + float((tb[2][n] - b).abs().max()), ef + float((fa[2][n] - b).abs().max()))
            b_max[n] = b_max.get(n, 0.0) + float(b.abs().max())
    assert e_out[1] <= 2 * e_out[0] + 1e-3 * len(seeds), ("logits", e_out)
    worse = [(n, ef, eb, g_norm[n]) for n, (eb, ef) in e_grad.items() if ef > 2 * eb + 1e-3 * g_norm[n] + 1e-12]
    assert not worse, worse
    if check_buffers:
        worse = [(n, ef, eb) for n, (eb, ef) in e_buf.items() if ef > 2 * eb + 1e-3 * b_max[n] + 1e-6]
        assert not worse, worse
