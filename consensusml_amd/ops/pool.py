"""NHWC bf16 max-pool with the HIP kernels of ``csrc/kernels/pool.hip`` (uint8 argmax, gather
backward), and the stem's BN + ReLU + max-pool fused so the BN output is never stored; other
inputs use ``F.max_pool2d`` / the unfused modules."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .native import lib


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, idx = lib().maxpool_fwd(x, k, s, p)
        ctx.save_for_backward(idx)
        ctx.geom = (x.shape[2], x.shape[3], k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        H, W, k, s, p = ctx.geom
        return lib().maxpool_bwd(dy, idx, H, W, k, s, p), None, None, None


def max_pool2d(x: torch.Tensor, k: int = 3, s: int = 2, p: int = 1) -> torch.Tensor:
    if (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0
            and (k + s - 1) // s <= 3 and k * k <= 255
            and x.is_contiguous(memory_format=torch.channels_last)):
        return _MaxPoolFn.apply(x, k, s, p)
    return F.max_pool2d(x, k, s, p)


def _pool_ok(x: torch.Tensor, k: int, s: int) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0
            and (k + s - 1) // s <= 3 and k * k <= 255
            and x.is_contiguous(memory_format=torch.channels_last))


class _BNReluPoolFn(torch.autograd.Function):
    """maxpool(relu(bn(x))): forward = BN statistics + ONE pass that applies the affine and ReLU
    to every window tap and keeps the max (the 112x112 BN output is never written); backward =
    the pool's gather into the BN-output gradient (ReLU-masked by the forward's argmax 255 for
    windows whose max is <= 0), then the fused BN backward."""

    @staticmethod
    def forward(ctx, x, gamma, beta, rmean, rvar, stats, eps, momentum, training, k, s, p):
        mi, ii = stats if stats is not None else (None, None)
        y, idx, mean, invstd = lib().bn_relu_maxpool_fwd(x, gamma, beta, rmean, rvar, mi, ii, eps,
                                                         momentum, training, k, s, p)
        ctx.save_for_backward(x, idx, gamma, beta, mean, invstd)
        ctx.geom = (k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, idx, gamma, beta, mean, invstd = ctx.saved_tensors
        k, s, p = ctx.geom
        dz = lib().maxpool_bwd(dy, idx, x.shape[2], x.shape[3], k, s, p)
        # the forward marked windows with max <= 0 (argmax 255): dz is already ReLU-masked
        dx, dg, db, _ = lib().bn_bwd(dz, None, x, None, gamma, beta, mean, invstd, False, False)
        return dx, dg, db, None, None, None, None, None, None, None, None, None


def bn_relu_max_pool2d(x: torch.Tensor, bn, k: int = 3, s: int = 2, p: int = 1) -> torch.Tensor:
    """``max_pool2d(bn(x))`` for a ReLU ``BatchNormAct2d`` ``bn``; fused on bf16 NHWC GPU tensors."""
    from .bn import _fused_ok
    if bn.relu and _pool_ok(x, k, s) and _fused_ok(x, bn.weight):
        stats = None
        if not bn.training:
            stats = (bn.running_mean.float(), torch.rsqrt(bn.running_var.float() + bn.eps))
        return _BNReluPoolFn.apply(x, bn.weight, bn.bias,
                                   bn.running_mean if bn.training else None,
                                   bn.running_var if bn.training else None, stats, bn.eps,
                                   bn.momentum, bn.training, k, s, p)
    return max_pool2d(bn(x), k, s, p)
