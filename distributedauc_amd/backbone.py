"""ResNet backbones with a 2-way softmax head (the score model of the reference).

The reference scores images with a torchvision-style ResNet whose head is
``Linear(512*expansion, 2)`` followed by ``Softmax(dim=1)`` (resnet.py:124-218):
the AUC score is column 1 of that softmax. This module builds the same
architectures (ResNet-18/34/50/101/152, ResNeXt-50/101, Wide-ResNet-50/101)
with the same parameter names, so a reference state_dict loads unchanged. The
convolutions run on PyTorch-ROCm (MIOpen / CK, hipBLASLt for the 1x1 GEMMs, bf16
autocast in the trainer). Switches put other passes on libdauc.so's HIP kernels:
set_fused_bn (bn + add + ReLU, csrc/bn_act.hip; the stem max-pool, csrc/maxpool.hip),
set_gemm_conv1x1 (conv1x1.py) and set_weight_shadow (one bf16 cast of all weights per
forward; the stride-1 3x3 input gradients as forward convolutions; the 3x3 weight
gradients, csrc/conv_wgrad.hip, and the 7x7 stem's forward and weight gradient,
csrc/conv_stem.hip, on MFMA kernels). Parity bars: BN vs fp64 torch (fp32 2e-5, bf16
2^-7 of scale), max-pool bit-identical to torch, weight gradients vs fp64 within 2e-5
of scale, the stem forward one bf16 rounding of the fp64 result (tests/test_*_gpu.py).

Pretrained weights are a network download in the reference (resnet.py:15-25,
228-237); this build has no network, so ``pretrained=True`` requires a local
state_dict path.
"""
from __future__ import annotations

import weakref

import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = [
    "ResNet", "resnet18", "resnet34", "resnet50", "resnet101", "resnet152", "resnext50_32x4d",
    "resnext101_32x8d", "wide_resnet50_2", "wide_resnet101_2", "build_backbone",
]


def _bn_act(fused: bool, bn: nn.BatchNorm2d, x: torch.Tensor, relu: bool = True,
            residual: torch.Tensor | None = None) -> torch.Tensor:
    """relu?(bn(x) + residual?): one fused HIP node when ``fused`` and training (fused_bn.py),
    torch's own modules otherwise (eval mode uses the running statistics)."""
    if fused and bn.training:
        from .fused_bn import bn_act

        return bn_act(x, bn, relu, residual)
    y = bn(x)
    if residual is not None:
        y = y + residual
    return F.relu(y, inplace=True) if relu else y


# ---- bf16 weight shadow ---------------------------------------------------------------------
# Under bf16 autocast every convolution casts its fp32 master weight to bf16 on every forward: one
# small cast launch per conv (ResNet-50: 53 launches, ~0.3 ms of a 26 ms step, each a few us of
# launch latency for a few hundred KB). With the shadow on, ONE cast launch per forward writes bf16
# copies of all parameters (the FlatState buffer is contiguous) and the convolutions read their
# bf16 weight from it: the same conversion (round to nearest even), so the same bits.
_shadow_live: list = []  # the shadow of the forward in flight (set by ResNet.features)


class WeightShadow:
    """bf16 copies of a FlatState's parameters at the same offsets (views per conv weight), and,
    with ``dgrad_fwd``, each stride-1 'same' k x k convolution's weight flipped and transposed
    (W'[ci, co, kh, kw] = W[co, ci, k-1-kh, k-1-kw], channels-last) for its input gradient.

    Two buffer sets, used by alternate forwards: the convolutions save views of the shadow for
    their backward, so refreshing the set a pending backward still holds would trip autograd's
    in-place check. With two, two grad-enabled forwards may precede one backward (summed losses
    over two micro-batches or two views); a third forward before that backward reuses the first
    set and autograd raises (never silently stale weights)."""

    def __init__(self, model: nn.Module, dgrad_fwd: bool = False, wgrad_hip: bool = False):
        flat = getattr(model, "_dauc_flat", None)
        if flat is None:
            raise RuntimeError("the weight shadow mirrors the FlatState buffer: build CoDA / FlatState first")
        self.src = flat.params
        self._model = weakref.ref(model)
        self.wgrad_hip = bool(wgrad_hip)
        dev = self.src.device
        convs = {id(m.weight): m for m in model.modules() if isinstance(m, nn.Conv2d)}
        idx, foff, vspec, fspec = [], 0, {}, {}
        for _, p, off, _n in flat.entries:
            m = convs.get(id(p))
            if m is None:
                continue
            vspec[id(p)] = (p.shape, p.stride(), off)
            if dgrad_fwd and _dgrad_as_fwd_ok(m):
                co, ci, k, _ = p.shape
                s0, s1, s2, s3 = p.stride()
                r = torch.arange(k)
                src = (off + torch.arange(co).view(1, co, 1, 1) * s0 + torch.arange(ci).view(ci, 1, 1, 1) * s1
                       + (k - 1 - r).view(1, 1, k, 1) * s2 + (k - 1 - r).view(1, 1, 1, k) * s3)  # [ci, co, kh, kw]
                idx.append(src.permute(0, 2, 3, 1).reshape(-1))  # channels-last storage order (ci, kh, kw, co)
                fspec[id(p)] = ((ci, co, k, k), (k * k * co, 1, k * co, co), foff)
                foff += p.numel()
        # int32 gather indices (ResNet-50: 11 M of them; int64 would double the bytes read per refresh)
        self.fidx = torch.cat(idx).to(device=dev, dtype=torch.int32) if idx else None
        self._sets = []
        for _ in range(2):
            buf = torch.empty(self.src.numel(), dtype=torch.bfloat16, device=dev)
            fbuf = torch.empty(foff, dtype=torch.bfloat16, device=dev) if foff else None
            views = {k: torch.as_strided(buf, sh, st, o) for k, (sh, st, o) in vspec.items()}
            flips = {k: torch.as_strided(fbuf, sh, st, o) for k, (sh, st, o) in fspec.items()}
            self._sets.append((buf, fbuf, views, flips))
        self._cur = 1
        self.buf, self.fbuf, self.views, self.flips = self._sets[0]

    def refresh(self, flips: bool = True) -> None:
        """Switch to the other buffer set, then one cast launch: bf16(params) -> the shadow
        (stream-ordered after the last update); with the flipped weights, one gather launch more."""
        m = self._model()
        flat = getattr(m, "_dauc_flat", None) if m is not None else None
        if flat is None or flat.params is not self.src:
            # a later FlatState moved the parameters into another buffer: this shadow would mirror
            # the old one and every bf16 forward would read stale weights
            raise RuntimeError("weight shadow is stale: the model's parameters moved to a new FlatState; call "
                               "model.set_weight_shadow(...) again after building it (CoDA does)")
        self._cur ^= 1
        self.buf, self.fbuf, self.views, self.flips = self._sets[self._cur]
        self.buf.copy_(self.src)
        if flips and self.fbuf is not None:
            torch.index_select(self.buf, 0, self.fidx, out=self.fbuf)

    def weight(self, p: torch.Tensor) -> torch.Tensor | None:
        return self.views.get(id(p))

    def flipped(self, p: torch.Tensor) -> torch.Tensor | None:
        return self.flips.get(id(p))


def _dgrad_as_fwd_ok(m: nn.Conv2d) -> bool:
    """A stride-1, 'same'-padded, odd square k x k convolution (k > 1, one group): its input
    gradient is the forward convolution of dy with the flipped, transposed weight."""
    k = m.kernel_size
    return (k[0] == k[1] and k[0] % 2 == 1 and k[0] > 1 and m.stride == (1, 1) and m.dilation == (1, 1)
            and m.groups == 1 and not isinstance(m.padding, str) and tuple(m.padding) == (k[0] // 2, k[0] // 2)
            and m.padding_mode == "zeros")


def shadow_weight(p: torch.Tensor, dtype: torch.dtype) -> torch.Tensor | None:
    """The bf16 shadow of conv weight ``p`` for the forward in flight, or None (cast it yourself)."""
    if not _shadow_live or dtype != torch.bfloat16:
        return None
    return _shadow_live[-1].weight(p)


class _ShadowConv(torch.autograd.Function):
    """conv2d(x, w_bf16) with the weight read from the shadow; the weight gradient goes to the fp32
    master weight exactly as autocast's graph sends it (aten.convolution_backward in bf16, then the
    bf16 -> fp32 copy of ToCopyBackward). The input gradient is torch's too, unless ``wf`` (the
    flipped weight) is given: then dx = conv2d(dy, wf) -- a FORWARD convolution of the same shape
    as this one (C_in = C_out for the bottlenecks' 3x3), which runs on the forward solvers (CK,
    no output zero-fill) instead of MIOpen's backward-data kernel and its zero-fill. Same
    products, fp32 accumulation in another order: the bits of dx differ from torch's. With
    ``wgrad_hip`` the 3x3 weight gradients come from csrc/conv_wgrad.hip and the 7x7 stem's forward
    and weight gradient from csrc/conv_stem.hip (fp32 gradients, no bf16 round trip)."""

    @staticmethod
    def forward(ctx, x, weight, wb, wf, stride, padding, dilation, groups, wgrad_hip=False):
        ctx.stem = False
        if wgrad_hip:
            from . import ops

            ctx.stem = ops.stem_conv_supported(x, wb, stride, padding, dilation, groups)
        if ctx.stem:  # the 7x7 stem on csrc/conv_stem.hip (MIOpen: ~6x the HBM-bound time)
            y = ops.stem_conv_forward(x, wb)
        else:
            with torch.autocast("cuda", enabled=False):
                y = F.conv2d(x, wb, None, stride, padding, dilation, groups)
        ctx.save_for_backward(x, wb, wf)
        ctx.conf = (list(stride), list(padding), list(dilation), groups)
        ctx.wgrad_hip = bool(wgrad_hip)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, wb, wf = ctx.saved_tensors
        stride, padding, dilation, groups = ctx.conf
        nx, nw = bool(ctx.needs_input_grad[0]), bool(ctx.needs_input_grad[1])
        dx = dw = None
        if nw and ctx.stem and gy.dtype == torch.bfloat16:
            from . import ops

            dw = ops.stem_conv_wgrad(x, gy.contiguous(memory_format=torch.channels_last))
        elif nw and ctx.wgrad_hip and wb.shape[2:] == (3, 3):
            from . import ops

            gyc = gy.contiguous(memory_format=torch.channels_last)
            if ops.conv3x3_wgrad_supported(x, gyc, stride, padding, dilation, groups):
                # the fp32 master gradient straight from csrc/conv_wgrad.hip (no bf16 round trip)
                dw = ops.conv3x3_wgrad(x, gyc, stride[0])
        mw = nw and dw is None
        if wf is not None and nx:
            dx = F.conv2d(gy.contiguous(memory_format=torch.channels_last), wf, None, 1, padding, 1, 1)
            if mw:
                dw = torch.ops.aten.convolution_backward(gy, x, wb, None, stride, padding, dilation, False, [0, 0],
                                                         groups, [False, True, False])[1].float()
        elif nx or mw:
            dx, dwb, _ = torch.ops.aten.convolution_backward(gy, x, wb, None, stride, padding, dilation, False,
                                                              [0, 0], groups, [nx, mw, False])
            if mw:
                dw = dwb.float()
        return dx, dw, None, None, None, None, None, None, None


def _cw(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """``conv(x)`` (a k x k convolution), reading its weight from the bf16 shadow when one is live."""
    wb = shadow_weight(conv.weight, torch.bfloat16) if x.is_cuda else None
    if (wb is None or conv.bias is not None or conv.padding_mode != "zeros" or isinstance(conv.padding, str)
            or not torch.is_autocast_enabled("cuda")):
        return conv(x)
    if x.dtype == torch.float32:
        x = x.to(torch.bfloat16)  # autocast's input cast
    if x.dtype != torch.bfloat16:
        return conv(x)
    sh = _shadow_live[-1]
    wf = sh.flipped(conv.weight) if torch.is_grad_enabled() else None
    return _ShadowConv.apply(x, conv.weight, wb, wf, conv.stride, conv.padding, conv.dilation, conv.groups,
                             sh.wgrad_hip)


class _GlobalAvgPoolCL(torch.autograd.Function):
    """adaptive_avg_pool2d(x, 1) of a channels-last activation with its gradient produced straight
    in channels-last. torch's backward (MeanBackward: grad.expand(x.shape) / (H*W)) writes an NCHW
    tensor that the fused BN backward then copies into channels-last: ResNet-50 b256, 2 passes over
    25.7 M elements, 0.11 ms per step, the transposing copy alone 85 us. Here the same division
    (the same elementwise op on the [N, C, 1, 1] gradient, so the same bits) is broadcast into a
    channels-last tensor by one copy."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        return F.adaptive_avg_pool2d(x, 1)

    @staticmethod
    def backward(ctx, g):
        N, C, H, W = ctx.shape
        gs = g / (H * W)
        if gs.is_cuda and gs.dtype == torch.bfloat16 and C % 8 == 0:
            from . import ops

            return ops.broadcast_hw(gs, H, W)  # csrc/strided.hip: the broadcast at HBM rate
        out = torch.empty((N, C, H, W), dtype=gs.dtype, device=gs.device, memory_format=torch.channels_last)
        out.copy_(gs.expand(N, C, H, W))
        return out


def _global_pool(pool: nn.Module, x: torch.Tensor) -> torch.Tensor:
    if (x.is_cuda and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)
            and isinstance(pool, nn.AdaptiveAvgPool2d) and pool.output_size in (1, (1, 1)) and torch.is_grad_enabled()):
        return _GlobalAvgPoolCL.apply(x)
    return pool(x)


def _c1(gemm: bool, conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """A 1x1 conv: through conv1x1.py (GEMM or MIOpen, timed per shape) when ``gemm``, else the module."""
    if gemm:
        from .conv1x1 import conv1x1

        return conv1x1(conv, x)
    return conv(x)


def _conv(cin: int, cout: int, k: int, stride: int = 1, groups: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, kernel_size=k, stride=stride, padding=k // 2, groups=groups, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, planes, stride=1, downsample=None, groups=1, base_width=64):
        super().__init__()
        if groups != 1 or base_width != 64:
            raise ValueError("BasicBlock supports groups=1, base_width=64 only")
        self.conv1 = _conv(cin, planes, 3, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = _conv(planes, planes, 3)
        self.bn2 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.fused_bn = False
        self.gemm_conv1x1 = False

    def forward(self, x):
        f = self.fused_bn
        skip = x if self.downsample is None else _bn_act(f, self.downsample[1], _c1(self.gemm_conv1x1,
                                                                                  self.downsample[0], x),
                                                         relu=False)
        y = _bn_act(f, self.bn1, _cw(self.conv1, x))
        return _bn_act(f, self.bn2, _cw(self.conv2, y), residual=skip)


class Bottleneck(nn.Module):
    """1x1 -> 3x3 (carries the stride) -> 1x1, x4 expansion."""

    expansion = 4

    def __init__(self, cin, planes, stride=1, downsample=None, groups=1, base_width=64):
        super().__init__()
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = _conv(cin, width, 1)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = _conv(width, width, 3, stride, groups)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = _conv(width, planes * self.expansion, 1)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.fused_bn = False
        self.gemm_conv1x1 = False

    def forward(self, x):
        f, g = self.fused_bn, self.gemm_conv1x1
        down = None if self.downsample is None else self.downsample[0]
        if g and x.is_cuda:
            # conv1 and the skip branch in one node: the gradient sum at x rides in the dgrad GEMM
            from .conv1x1 import conv1x1_skip

            h, skip = conv1x1_skip(self.conv1, x, down, skip_grad_owned=f and self.training)
        else:
            h, skip = _c1(g, self.conv1, x), (x if down is None else _c1(g, down, x))
        if down is not None:
            skip = _bn_act(f, self.downsample[1], skip, relu=False)
        y = _bn_act(f, self.bn1, h)
        y = _bn_act(f, self.bn2, _cw(self.conv2, y))
        return _bn_act(f, self.bn3, _c1(g, self.conv3, y), residual=skip)


class ResNet(nn.Module):
    """Stem (7x7/2 conv, BN, ReLU, 3x3/2 max-pool) -> 4 stages -> avg-pool -> fc -> softmax."""

    def __init__(self, block, layers, num_classes: int = 2, groups: int = 1, width_per_group: int = 64,
                 zero_init_residual: bool = False, head: str = "softmax"):
        super().__init__()
        if head not in ("softmax", "logits"):
            raise ValueError("head must be 'softmax' or 'logits'")
        self.groups = groups
        self.base_width = width_per_group
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._stage(block, 64, layers[0], 1)
        self.layer2 = self._stage(block, 128, layers[1], 2)
        self.layer3 = self._stage(block, 256, layers[2], 2)
        self.layer4 = self._stage(block, 512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        # "logits": the surrogate kernel applies the softmax column itself
        self.softmax = nn.Softmax(dim=1) if head == "softmax" else nn.Identity()
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def _stage(self, block, planes, blocks, stride):
        down = None
        cout = planes * block.expansion
        if stride != 1 or self.inplanes != cout:
            down = nn.Sequential(_conv(self.inplanes, cout, 1, stride), nn.BatchNorm2d(cout))
        mods = [block(self.inplanes, planes, stride, down, self.groups, self.base_width)]
        self.inplanes = cout
        mods += [block(cout, planes, 1, None, self.groups, self.base_width) for _ in range(1, blocks)]
        return nn.Sequential(*mods)

    fused_bn = False
    _counted_bns: list = []
    _wshadow: WeightShadow | None = None

    def set_weight_shadow(self, enabled: bool = True, dgrad_fwd: bool = True, wgrad_hip: bool = True) -> "ResNet":
        """Read every convolution's bf16 weight from one shadow buffer refreshed by a single cast
        launch per forward, instead of autocast's cast per convolution (bf16 autocast only; the
        parameters must already live in a FlatState, i.e. after CoDA(model)). ``dgrad_fwd``: the
        stride-1 3x3 convolutions' input gradients as forward convolutions with flipped weights
        (_ShadowConv). ``wgrad_hip``: the 3x3 weight gradients from csrc/conv_wgrad.hip (fp32, MFMA)
        instead of MIOpen's backward-weights + the bf16 -> fp32 cast, and the 7x7 stem's forward
        and weight gradient from csrc/conv_stem.hip."""
        self._wshadow = WeightShadow(self, dgrad_fwd=dgrad_fwd, wgrad_hip=wgrad_hip) if enabled else None
        return self

    def set_fused_bn(self, enabled: bool = True) -> "ResNet":
        """Route every training-mode bn (+ add) + relu through the fused HIP kernels (channels-last
        bf16/fp32 on the GPU; csrc/bn_act.hip). Parameter and buffer names are unchanged."""
        self.fused_bn = bool(enabled)
        self._counted_bns = []
        for m in self.modules():
            if isinstance(m, (BasicBlock, Bottleneck)):
                m.fused_bn = self.fused_bn
            if isinstance(m, nn.BatchNorm2d):
                # fused training forwards bump every BN's num_batches_tracked in ONE multi-tensor
                # launch (features()) instead of one add kernel per layer; momentum=None layers
                # need the count inside their own node and keep counting there
                batched = self.fused_bn and m.track_running_stats and m.momentum is not None
                m._dauc_counted = batched
                if batched:
                    self._counted_bns.append(m)
        return self

    def set_gemm_conv1x1(self, enabled: bool = True) -> "ResNet":
        """Run the stride-1 1x1 convolutions as GEMMs where that is faster (conv1x1.py; channels-last GPU)."""
        for m in self.modules():
            if isinstance(m, (BasicBlock, Bottleneck)):
                m.gemm_conv1x1 = bool(enabled)
        return self

    def features(self, x):
        if self.fused_bn and self.training and x.is_cuda and self._counted_bns:
            torch._foreach_add_([m.num_batches_tracked for m in self._counted_bns], 1)
        live = (self._wshadow is not None and x.is_cuda and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.bfloat16)
        if live:
            self._wshadow.refresh(flips=torch.is_grad_enabled())
            _shadow_live.append(self._wshadow)
        try:
            x = _bn_act(self.fused_bn, self.bn1, _cw(self.conv1, x))
            if self.fused_bn and x.is_cuda:  # the stem max-pool with int8 indices (pool.py)
                from .pool import max_pool2d

                x = max_pool2d(x, self.maxpool)
            else:
                x = self.maxpool(x)
            x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        finally:
            if live:
                _shadow_live.pop()
        return torch.flatten(_global_pool(self.avgpool, x), 1)

    def forward(self, x):
        return self.softmax(self.fc(self.features(x)))


_SPECS = {
    "resnet18": (BasicBlock, [2, 2, 2, 2], {}),
    "resnet34": (BasicBlock, [3, 4, 6, 3], {}),
    "resnet50": (Bottleneck, [3, 4, 6, 3], {}),
    "resnet101": (Bottleneck, [3, 4, 23, 3], {}),
    "resnet152": (Bottleneck, [3, 8, 36, 3], {}),
    "resnext50_32x4d": (Bottleneck, [3, 4, 6, 3], {"groups": 32, "width_per_group": 4}),
    "resnext101_32x8d": (Bottleneck, [3, 4, 23, 3], {"groups": 32, "width_per_group": 8}),
    "wide_resnet50_2": (Bottleneck, [3, 4, 6, 3], {"width_per_group": 128}),
    "wide_resnet101_2": (Bottleneck, [3, 4, 23, 3], {"width_per_group": 128}),
}


def build_backbone(arch: str, pretrained: bool | str = False, **kwargs) -> ResNet:
    """Build ``arch``; ``pretrained`` may be a local state_dict path (fc.* is dropped, resnet.py:234-235)."""
    block, layers, extra = _SPECS[arch]
    model = ResNet(block, layers, **{**extra, **kwargs})
    if pretrained:
        if pretrained is True:
            raise RuntimeError("pretrained weights need a local state_dict path (no network in this build)")
        sd = torch.load(pretrained, map_location="cpu", weights_only=True)
        sd = {k: v for k, v in sd.items() if not k.startswith("fc.")}
        model.load_state_dict(sd, strict=False)
    return model


def _factory(name):
    def make(pretrained=False, progress=True, **kwargs):  # signature of resnet.py factories
        return build_backbone(name, pretrained, **kwargs)

    make.__name__ = name
    make.__doc__ = f"{name} with a 2-way softmax head (resnet.py factory of the same name)."
    return make


resnet18 = _factory("resnet18")
resnet34 = _factory("resnet34")
resnet50 = _factory("resnet50")
resnet101 = _factory("resnet101")
resnet152 = _factory("resnet152")
resnext50_32x4d = _factory("resnext50_32x4d")
resnext101_32x8d = _factory("resnext101_32x8d")
wide_resnet50_2 = _factory("wide_resnet50_2")
wide_resnet101_2 = _factory("wide_resnet101_2")
