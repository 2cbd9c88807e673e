"""The bf16 weight shadow (backbone.WeightShadow): one cast launch per forward instead of autocast's
cast per convolution must change no bit of the step; the 3x3 input gradients as forward
convolutions with flipped weights (dgrad_fwd) change only the summation order.

Reference: the same backbone under torch's bf16 autocast (main.py:311-326's forward/backward, the
autocast the trainer adds), where each conv casts its fp32 weight itself. Same model, same input,
deterministic MIOpen solvers and the GEMM engine fixed for the 1x1 convolutions (engine timing must
not pick different numerics for the two runs): scores, every parameter gradient and the loss after
a CoDA step are bit-identical with and without the shadow, and a parameter change between
forwards is seen by the next forward (the shadow is refreshed per forward).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bits(t):
    t = t.detach().contiguous()
    return t.view(torch.int16 if t.element_size() == 2 else torch.int32).cpu()


def _run(dev, arch, shadow, size, dgrad_fwd=False, autocast=True):
    from distributedauc_amd import conv1x1
    from distributedauc_amd.backbone import build_backbone
    from distributedauc_amd.coda import CoDA

    torch.manual_seed(7)
    net = build_backbone(arch, num_classes=2).to(dev).to(memory_format=torch.channels_last)
    net.set_fused_bn(True).set_gemm_conv1x1(True).train()
    coda = CoDA(net, lr=0.01, split_index=4, autocast_dtype=torch.bfloat16 if autocast else None, device=dev,
                weight_shadow=shadow)
    assert (net._wshadow is not None) == shadow
    if shadow and not dgrad_fwd:
        net.set_weight_shadow(True, dgrad_fwd=False, wgrad_hip=False)  # torch's backward: bit-identical
    g = torch.Generator(device=dev).manual_seed(11)
    x = torch.randn((8, 3, size, size), device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.tensor([9, 0, 7, 1, 5, 3, 8, 2], device=dev)
    with conv1x1.fixed_engine("gemm"):
        h = coda.scores(x)
        h.float().pow(2).sum().backward()
        grads = [p.grad.detach().clone() for p in net.parameters()]
        net.zero_grad(set_to_none=True)
        loss = coda.train_step(x, y)  # forward, surrogate, backward, update
        coda.state.params.mul_(0.5)   # parameters change between forwards: the shadow must follow
        h2 = coda.scores(x)
    return h.detach().clone(), grads, float(loss), h2.detach().clone(), coda.state.flat.clone()


@pytest.mark.parametrize("arch,size", [("resnet18", 64), ("resnet50", 64)])
def test_weight_shadow_bit_identical(dev, arch, size):
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        a = _run(dev, arch, False, size)
        b = _run(dev, arch, True, size)
    finally:
        torch.backends.cudnn.deterministic = det
    assert torch.equal(_bits(a[0]), _bits(b[0])), "scores differ"
    assert len(a[1]) == len(b[1])
    for i, (ga, gb) in enumerate(zip(a[1], b[1])):
        assert torch.equal(_bits(ga), _bits(gb)), f"gradient {i} differs"
    assert a[2] == b[2] or (a[2] != a[2] and b[2] != b[2]), "loss differs"
    assert torch.equal(_bits(a[3]), _bits(b[3])), "scores after a parameter change differ"
    assert torch.equal(_bits(a[4]), _bits(b[4])), "state after the step differs"


def test_weight_shadow_needs_flat_state(dev):
    from distributedauc_amd.backbone import resnet18

    net = resnet18().to(dev)
    with pytest.raises(RuntimeError, match="FlatState"):
        net.set_weight_shadow(True)


def _rel_excess(got, ref):
    """max over elements of (|got - ref| - |ref| * 2^-8) / max|ref|: <= ~0 when got is ref rounded
    once to bf16 (an fp32-accumulated sum rounded once)."""
    err = (got.double() - ref).abs()
    return float((err - ref.abs() * 2 ** -8).max() / ref.abs().max())


@pytest.mark.parametrize("shape", [(4, 64, 56, 56), (4, 128, 28, 28), (8, 512, 7, 7), (2, 24, 9, 13)])
def test_dgrad_as_forward_conv(dev, shape):
    """_ShadowConv with the flipped weight: dx = conv2d(dy, W') against the fp64 result of the same
    bf16 operands: one bf16 rounding of an fp32 sum (the forward solvers accumulate in fp32). torch's
    backward-data on the same operands is reported beside it (MIOpen's split accumulation may round
    more than once). Forward output and weight gradient: the same calls, bit-identical under
    deterministic solvers."""
    from distributedauc_amd.backbone import _ShadowConv

    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        N, C, H, W = shape
        g = torch.Generator(device=dev).manual_seed(5)
        x = torch.randn(shape, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn((C, C, 3, 3), device=dev, generator=g) / (3 * C ** 0.5)).to(torch.bfloat16)
        w = w.contiguous(memory_format=torch.channels_last)
        wf = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)
        gy = torch.randn(shape, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        p = torch.zeros((C, C, 3, 3), device=dev, requires_grad=True)
        xa = x.clone().requires_grad_(True)
        ya = _ShadowConv.apply(xa, p, w, wf, (1, 1), (1, 1), (1, 1), 1)
        ya.backward(gy)
        xb = x.clone().requires_grad_(True)
        pb = torch.zeros((C, C, 3, 3), device=dev, requires_grad=True)
        yb = _ShadowConv.apply(xb, pb, w, None, (1, 1), (1, 1), (1, 1), 1)
        yb.backward(gy)
    finally:
        torch.backends.cudnn.deterministic = det
    assert torch.equal(ya, yb)
    assert torch.equal(p.grad, pb.grad)
    assert xa.grad.is_contiguous(memory_format=torch.channels_last)
    ref = torch.nn.functional.conv2d(gy.double(), wf.double(), padding=1)
    ours, theirs = _rel_excess(xa.grad, ref), _rel_excess(xb.grad, ref)
    assert ours <= 1e-5, (ours, theirs)


def test_weight_shadow_dgrad_fwd_step_close(dev):
    """The whole ResNet-50 step with the HIP convolution paths (dgrad_fwd, the 3x3 weight gradients,
    the 7x7 stem's forward and weight gradient) against torch's, both against the fp32 step (no
    autocast): scores and every gradient are as close to fp32 as torch's bf16 step is (bf16
    rounding differences propagate through 50 layers, so the two bf16 steps differ from each other
    by about as much as each differs from fp32)."""
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        ref = _run(dev, "resnet50", False, 64, autocast=False)
        a = _run(dev, "resnet50", True, 64, dgrad_fwd=False)
        b = _run(dev, "resnet50", True, 64, dgrad_fwd=True)
    finally:
        torch.backends.cudnn.deterministic = det
    sa, sb = float((a[0].float() - ref[0].float()).abs().max()), float((b[0].float() - ref[0].float()).abs().max())
    assert sb <= 2.0 * sa + 1e-2, (sb, sa)
    ea, eb = [], []
    for g32, ga, gb in zip(ref[1], a[1], b[1]):
        scale = float(g32.abs().max().clamp_min(1e-30))
        ea.append(float((ga - g32).abs().max()) / scale)
        eb.append(float((gb - g32).abs().max()) / scale)
    ea, eb = np.array(ea), np.array(eb)
    assert np.median(eb) <= 1.5 * np.median(ea) + 1e-3, (np.median(eb), np.median(ea))
    assert eb.max() <= 2.0 * ea.max() + 1e-2, (eb.max(), ea.max())


def test_nchw_model_channels_last_input_default_coda(dev):
    """an NCHW model (build_backbone's default) fed channels-last images under default
    CoDA (bf16 autocast: the shadow and the HIP weight-gradient paths on) trains: the stem kernels
    take only a channels-last bf16 weight, so the stem falls back to F.conv2d instead of raising."""
    from distributedauc_amd import ops
    from distributedauc_amd.backbone import build_backbone
    from distributedauc_amd.coda import CoDA

    torch.manual_seed(3)
    net = build_backbone("resnet18", num_classes=2).to(dev).set_fused_bn(True).train()
    coda = CoDA(net, lr=0.01, split_index=4, autocast_dtype=torch.bfloat16, device=dev)
    assert net._wshadow is not None and net._wshadow.wgrad_hip
    wb = net._wshadow.weight(net.conv1.weight)
    assert not ops.stem_conv_supported(torch.zeros((2, 3, 32, 32), device=dev, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last), wb, (2, 2), (3, 3), (1, 1), 1)
    g = torch.Generator(device=dev).manual_seed(2)
    x = torch.randn((8, 3, 32, 32), device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.tensor([9, 0, 7, 1, 5, 3, 8, 2], device=dev)
    loss = coda.train_step(x, y)
    loss2 = coda.train_step(x, y)
    torch.cuda.synchronize()
    assert np.isfinite(float(loss)) and np.isfinite(float(loss2))
    assert bool(torch.isfinite(coda.state.flat).all())


def test_shadow_follows_new_flat_state(dev):
    """a second CoDA on the same model moves the parameters into a new FlatState; its
    weight_shadow=False must turn the old shadow off, and a shadow left mirroring an old buffer
    raises at the next forward instead of reading stale weights."""
    from distributedauc_amd.backbone import build_backbone
    from distributedauc_amd.coda import CoDA
    from distributedauc_amd.flat import FlatState

    torch.manual_seed(4)
    net = build_backbone("resnet18", num_classes=2).to(dev).to(memory_format=torch.channels_last)
    net.set_fused_bn(True).train()
    CoDA(net, lr=0.01, split_index=4, autocast_dtype=torch.bfloat16, device=dev)
    assert net._wshadow is not None
    CoDA(net, lr=0.01, split_index=4, autocast_dtype=torch.bfloat16, device=dev, weight_shadow=False)
    assert net._wshadow is None
    coda = CoDA(net, lr=0.01, split_index=4, autocast_dtype=torch.bfloat16, device=dev)
    assert net._wshadow is not None and net._wshadow.src is coda.state.params
    FlatState(net, dev)  # parameters move again, the shadow is not rebuilt
    x = torch.randn((4, 3, 32, 32), device=dev).contiguous(memory_format=torch.channels_last)
    with pytest.raises(RuntimeError, match="stale"):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            net(x)


def test_two_forwards_one_backward(dev):
    """two grad-enabled forwards before one backward (a loss summed over two
    micro-batches) work with the shadow on -- each forward refreshes the other buffer set, so the
    views the first forward saved are intact -- and give the same gradients, bit for bit, as the
    same two forwards without the shadow (torch's backward: dgrad_fwd and wgrad_hip off,
    deterministic solvers, the GEMM engine fixed)."""
    from distributedauc_amd import conv1x1
    from distributedauc_amd.backbone import build_backbone
    from distributedauc_amd.coda import CoDA

    def run(shadow):
        torch.manual_seed(8)
        net = build_backbone("resnet18", num_classes=2).to(dev).to(memory_format=torch.channels_last)
        net.set_fused_bn(True).set_gemm_conv1x1(True).train()
        coda = CoDA(net, lr=0.01, split_index=4, autocast_dtype=torch.bfloat16, device=dev, weight_shadow=shadow)
        if shadow:
            net.set_weight_shadow(True, dgrad_fwd=False, wgrad_hip=False)
        g = torch.Generator(device=dev).manual_seed(12)
        x1 = torch.randn((4, 3, 32, 32), device=dev, generator=g).contiguous(memory_format=torch.channels_last)
        x2 = torch.randn((4, 3, 32, 32), device=dev, generator=g).contiguous(memory_format=torch.channels_last)
        with conv1x1.fixed_engine("gemm"):
            loss = coda.scores(x1).pow(2).sum() + coda.scores(x2).sum()
            loss.backward()
        return [p.grad.detach().clone() for p in net.parameters()]

    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        a, b = run(False), run(True)
    finally:
        torch.backends.cudnn.deterministic = det
    for i, (ga, gb) in enumerate(zip(a, b)):
        assert torch.equal(_bits(ga), _bits(gb)), f"gradient {i} differs"
