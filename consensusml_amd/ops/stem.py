"""ResNet stem ``maxpool(relu(bn(conv7x7_s2(x))))`` as two HIP passes each way
(``csrc/kernels/stem_conv.hip`` + the BN-affine max-pool of ``pool.hip``).

forward : MFMA implicit-GEMM conv that also accumulates the BN statistics (no statistics pass,
          no channel-padding pass for 3-channel images), then the pool that applies BN + ReLU to
          every window tap (the BN output is never stored).
backward: ONE MFMA pass that produces the conv weight gradient through the BatchNorm plus dgamma
          (the BN input gradient is never formed; see the kernel header for the algebra), reading
          the pool's OUTPUT gradient: each pixel's pool input gradient (ReLU-masked by the
          forward's argmax) is gathered from the windows that contain it while staging, after a
          small pass for its channel sums (= dbeta). PerfPolicy.stem_pool_gather off: the pool
          backward writes the full-resolution gradient (4x the pooled size) and the MFMA pass
          reads it back.

Other inputs (CPU, fp32, other stem shapes, images that need an input gradient, eval-mode
backward) take the module path.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..perf import policy as _P
from .native import lib


def pack_stem_weight(w: torch.Tensor) -> torch.Tensor:
    """[64, C, 7, 7] -> bf16 [64, 224], k = (ky * 8 + kx) * 4 + c (kx = 7 and c >= C zero)."""
    c = w.shape[1]
    wp = w.detach().to(torch.bfloat16).permute(0, 2, 3, 1)          # [64, 7, 7, C]
    return F.pad(wp, (0, 4 - c, 0, 1)).reshape(64, 224).contiguous()


class _StemFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, gamma, beta, rmean, rvar, eps, momentum, training, link=None):
        wpk = pack_stem_weight(weight)
        z, mean, invstd = lib().stem_conv_fwd(x, wpk, rmean if training else None,
                                              rvar if training else None, eps, momentum, training)
        if not training:
            mean = rmean.float().contiguous()
            invstd = torch.rsqrt(rvar.float() + eps).contiguous()
        y, idx, _, _ = lib().bn_relu_maxpool_fwd(z, gamma, beta, None, None, mean, invstd, eps,
                                                 momentum, False, 3, 2, 1)
        ctx.save_for_backward(x, z, idx, gamma, mean, invstd)
        ctx.dtypes = (weight.dtype, gamma.dtype, beta.dtype)
        ctx.link = link
        return y

    @staticmethod
    def backward(ctx, dy):
        x, z, idx, gamma, mean, invstd = ctx.saved_tensors
        # a second gradient of y parked by a link_tap consumer (layer1.0's downsample conv) is
        # summed inside the pool backward instead of by an autograd add
        dy2 = ctx.link.take_tensor() if ctx.link is not None else None
        if dy2 is not None and dy2.shape != dy.shape:
            dy, dy2 = dy + dy2, None
        wt, gt, bt = ctx.dtypes
        if _P().stem_pool_gather:
            # bf16 parameters: the final kernel writes bf16 itself (no three cast launches)
            bf = wt == gt == bt == torch.bfloat16
            dw, dg, db = lib().stem_wgrad_pool(dy, idx, dy2, z, x, mean, invstd, gamma, bf)
        else:
            g, gsum = lib().maxpool_bwd_sum(dy, idx, z.shape[2], z.shape[3], dy2)
            dw, dg, db = lib().stem_wgrad(g, z, x, mean, invstd, gamma, gsum)
        return None, dw.to(wt), dg.to(gt), db.to(bt), None, None, None, None, None, None


def stem_ok(x: torch.Tensor, conv, bn) -> bool:
    w = conv.weight
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] in (3, 4)
            and x.is_contiguous(memory_format=torch.channels_last) and not x.requires_grad
            and tuple(w.shape) == (64, x.shape[1], 7, 7) and conv.bias is None
            and tuple(conv.stride) == (2, 2) and tuple(conv.padding) == (3, 3)
            and tuple(conv.dilation) == (1, 1) and conv.groups == 1
            and (x.shape[3] - 1) // 2 + 1 <= 143 and bn.relu and bn.weight is not None
            and bn.weight.dtype == torch.bfloat16 and bn.bias.dtype == torch.bfloat16
            and bn.running_mean is not None
            and (bn.training or not (torch.is_grad_enabled() and w.requires_grad)))


def stem_conv_bn_relu_pool(x: torch.Tensor, conv, bn, link=None) -> torch.Tensor:
    """``max_pool2d(bn(conv(x)), 3, 2, 1)`` for the ResNet stem (``bn`` a ReLU BatchNormAct2d).
    ``link`` (ops.bn.ResidualLink): a consumer of the output may park a second output gradient
    there (ops.bn.link_tap); the backward sums it on load."""
    return _StemFn.apply(x, conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                         bn.eps, bn.momentum, bn.training, link)
