"""ResNet-50 (He et al. 2016, v1.5: stride on the 3x3 conv) for the headline benchmark (N12).

Convolutions run on MIOpen in bf16 with channels_last activations and weights (NHWC is MIOpen's
fast layout on CDNA). Every BatchNorm is a ``BatchNormAct2d``: BN + (residual add) + ReLU fused
into the HIP kernels of ``csrc/kernels/bn_act.hip`` on GPU — the block tail
``relu(bn3(conv3(x)) + identity)`` is one op. Random-init weights (no checkpoints offline).
BASELINE.json config: "ResNet-50 bf16 DP=8 with Krum".
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.bn import BatchNormAct2d, ResidualLink, fused_ok
from ..ops.pool import max_pool2d

# 1x1 stride-1 convolutions as plain GEMMs (see Conv1x1); toggled by bench.py --conv1x1.
# Off by default: measured on MI355X at batch 512 the hipBLASLt kernels chosen for these
# tall-skinny shapes (e.g. dW with K = N*H*W = 1.6M and a 64x64 output tile grid of 4) made the
# step 77 ms vs 55 ms with MIOpen's 1x1 solvers (profiles/r01_bench8_conv1x1_gemm_kernels.md).
CONV1X1_GEMM = os.environ.get("CML_CONV1X1_GEMM", "0") == "1"
# identity blocks fuse the residual-gradient add into conv1's dX GEMM (see ops.bn.ResidualLink)
RESIDUAL_LINK = True


class _Conv1x1Fn(torch.autograd.Function):
    """y = x W^T on [M, Cin] rows; backward dX = dY W accumulated into a linked residual
    gradient when one is parked (ResidualLink), dW = dY^T X."""

    @staticmethod
    def forward(ctx, x2d, w2d, link):
        ctx.save_for_backward(x2d, w2d)
        ctx.link = link
        return torch.mm(x2d, w2d.t())

    @staticmethod
    def backward(ctx, dy):
        x2d, w2d = ctx.saved_tensors
        dx = None
        if ctx.needs_input_grad[0]:
            link = ctx.link
            if link is not None and link.grad is not None:
                g = link.grad
                link.grad = None
                dres = g.permute(0, 2, 3, 1).reshape(dy.shape[0], -1) if g.dim() == 4 else g
                if dres.data_ptr() == g.data_ptr() and dres.is_contiguous():
                    dx = dres.addmm_(dy, w2d)          # beta = 1 GEMM epilogue, in place
                else:
                    dx = torch.addmm(dres, dy, w2d)
            else:
                dx = torch.mm(dy, w2d)
        dw = torch.mm(dy.t(), x2d) if ctx.needs_input_grad[1] else None
        return dx, dw, None


class Conv1x1(nn.Conv2d):
    """1x1 convolution. With stride 1 on a channels_last GPU tensor, the NHWC activation IS a
    row-major [N*H*W, C] matrix, so the conv is one GEMM (``F.linear`` -> hipBLASLt) and its
    backward two more (dX = dY W, dW = dY^T X) — no im2col, no layout change, output already
    channels_last. These are 8/17 of a bottleneck's FLOPs. Strided 1x1 (downsample) convs and CPU
    tensors use the regular MIOpen / ATen convolution. Same parameter as nn.Conv2d."""

    def __init__(self, cin: int, cout: int, stride: int = 1):
        super().__init__(cin, cout, 1, stride=stride, bias=False)

    def gemm_ok(self, x: torch.Tensor) -> bool:
        return (CONV1X1_GEMM and self.stride == (1, 1) and x.is_cuda
                and x.is_contiguous(memory_format=torch.channels_last))

    def forward(self, x: torch.Tensor, res_link: Optional[ResidualLink] = None) -> torch.Tensor:
        if self.gemm_ok(x):
            N, C, H, W = x.shape
            y = _Conv1x1Fn.apply(x.permute(0, 2, 3, 1).reshape(N * H * W, C),
                                 self.weight.reshape(self.out_channels, C), res_link)
            return y.view(N, H, W, self.out_channels).permute(0, 3, 1, 2)
        return super().forward(x)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: bool = False):
        super().__init__()
        self.conv1 = Conv1x1(inplanes, planes)
        self.bn1 = BatchNormAct2d(planes, relu=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = BatchNormAct2d(planes, relu=True)
        self.conv3 = Conv1x1(planes, planes * 4)
        self.bn3 = BatchNormAct2d(planes * 4, relu=True)      # + residual, fused
        if downsample:
            self.down_conv = Conv1x1(inplanes, planes * 4, stride=stride)
            self.down_bn = BatchNormAct2d(planes * 4, relu=False)
        else:
            self.down_conv = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        use_links = RESIDUAL_LINK and torch.is_grad_enabled() and self.training
        if self.down_conv is None:
            # identity block: bn3's residual gradient is parked on the link of our input (made by
            # the producing block); conv1's GEMM backward (if used) or the producer's BN backward
            # consumes it (see ops.bn.ResidualLink)
            link = getattr(x, "_cml_link", None) if use_links else None
            out = self.bn1(self.conv1(x, res_link=link if self.conv1.gemm_ok(x) else None))
            out = self.bn2(self.conv2(out))
            z = self.conv3(out)
            fused = fused_ok(z, self.bn3.weight)
            out_link = ResidualLink() if use_links and fused else None
            y = self.bn3(z, residual=x, res_link=link if fused else None, out_link=out_link)
        else:
            idt = self.down_bn(self.down_conv(x))
            out = self.bn1(self.conv1(x))
            out = self.bn2(self.conv2(out))
            z = self.conv3(out)
            out_link = ResidualLink() if use_links and fused_ok(z, self.bn3.weight) else None
            y = self.bn3(z, residual=idt, out_link=out_link)
        if out_link is not None:
            y._cml_link = out_link      # our consumer (an identity block) parks dres here
        return y


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
