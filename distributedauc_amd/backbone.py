"""ResNet backbones with a 2-way softmax head (the score model of the reference).

The reference scores images with a torchvision-style ResNet whose head is
``Linear(512*expansion, 2)`` followed by ``Softmax(dim=1)`` (resnet.py:124-218):
the AUC score is column 1 of that softmax. This module builds the same
architectures (ResNet-18/34/50/101/152, ResNeXt-50/101, Wide-ResNet-50/101)
with the same parameter names, so a reference state_dict loads unchanged. The
backbone runs on PyTorch-ROCm (MIOpen convolutions, bf16 autocast in the
trainer); only the AUC-specific work is in the HIP library.

Pretrained weights are a network download in the reference (resnet.py:15-25,
228-237); this build has no network, so ``pretrained=True`` requires a local
state_dict path.
"""
from __future__ import annotations

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
        y = _bn_act(f, self.bn1, self.conv1(x))
        return _bn_act(f, self.bn2, self.conv2(y), residual=skip)


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
        y = _bn_act(f, self.bn2, self.conv2(y))
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
        x = _bn_act(self.fused_bn, self.bn1, self.conv1(x))
        if self.fused_bn and x.is_cuda:  # the stem max-pool with int8 indices (pool.py)
            from .pool import max_pool2d

            x = max_pool2d(x, self.maxpool)
        else:
            x = self.maxpool(x)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return torch.flatten(self.avgpool(x), 1)

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
