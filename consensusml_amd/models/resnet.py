"""ResNet-50 (He et al. 2016, v1.5: stride on the 3x3 conv) for the headline benchmark (N12).

Convolutions run on MIOpen in bf16 with channels_last activations and weights (NHWC is MIOpen's
fast layout on CDNA). Every BatchNorm is a ``BatchNormAct2d``: BN + (residual add) + ReLU fused
into the HIP kernels of ``csrc/kernels/bn_act.hip`` on GPU — the block tail
``relu(bn3(conv3(x)) + identity)`` is one op. Random-init weights (no checkpoints offline).
BASELINE.json config: "ResNet-50 bf16 DP=8 with Krum".
"""
from __future__ import annotations

from typing import List

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.bn import BatchNormAct2d
from ..ops.pool import max_pool2d


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: bool = False):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = BatchNormAct2d(planes, relu=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = BatchNormAct2d(planes, relu=True)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = BatchNormAct2d(planes * 4, relu=True)      # + residual, fused
        if downsample:
            self.down_conv = nn.Conv2d(inplanes, planes * 4, 1, stride=stride, bias=False)
            self.down_bn = BatchNormAct2d(planes * 4, relu=False)
        else:
            self.down_conv = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        idt = x if self.down_conv is None else self.down_bn(self.down_conv(x))
        out = self.bn1(self.conv1(x))
        out = self.bn2(self.conv2(out))
        return self.bn3(self.conv3(out), residual=idt)


class ResNet(nn.Module):
    def __init__(self, layers: List[int], num_classes: int = 1000, width: int = 64):
        super().__init__()
        self.inplanes = width
        self.conv1 = nn.Conv2d(3, width, 7, stride=2, padding=3, bias=False)
        self.bn1 = BatchNormAct2d(width, relu=True)
        self.layer1 = self._make(width, layers[0], 1)
        self.layer2 = self._make(width * 2, layers[1], 2)
        self.layer3 = self._make(width * 4, layers[2], 2)
        self.layer4 = self._make(width * 8, layers[3], 2)
        self.fc = nn.Linear(width * 8 * 4, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        for m in self.modules():   # zero-init the last BN of each block (standard trick)
            if isinstance(m, Bottleneck):
                nn.init.zeros_(m.bn3.weight)

    def _make(self, planes: int, blocks: int, stride: int) -> nn.Sequential:
        down = stride != 1 or self.inplanes != planes * 4
        mods = [Bottleneck(self.inplanes, planes, stride, down)]
        self.inplanes = planes * 4
        mods += [Bottleneck(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*mods)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.bn1(self.conv1(x))
        x = max_pool2d(x, 3, 2, 1)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
        return self.fc(x)


def resnet50(num_classes: int = 1000) -> ResNet:
    return ResNet([3, 4, 6, 3], num_classes)


def resnet_tiny(num_classes: int = 10) -> ResNet:
    """Same block structure at width 8 / one block per stage (tests)."""
    return ResNet([1, 1, 1, 1], num_classes, width=8)
