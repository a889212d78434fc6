"""NHWC bf16 max-pool with the HIP kernels of ``csrc/kernels/pool.hip`` (uint8 argmax, gather
backward); other inputs use ``F.max_pool2d``."""
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
