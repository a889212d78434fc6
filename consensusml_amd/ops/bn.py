"""BatchNormAct2d: training BatchNorm + optional residual add + optional ReLU as one op.

GPU bf16 channels_last inputs run the fused HIP kernels of ``csrc/kernels/bn_act.hip``
(forward: stats + apply; backward: reduce + apply; the ReLU mask is recomputed from x, or — with a
residual — kept from the forward as one bit per element). Anything else (CPU tests,
fp32, NCHW) runs the equivalent PyTorch composition. Running statistics are kept in fp32 even
when the module is cast to bf16.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..perf import policy as _P
from .native import lib


class ResidualLink:
    """Hand-off of a residual gradient between the two consumers of a ResNet block input.

    A block input x (= the previous block's output y) feeds conv1 and the residual add of the
    block's last BN. Autograd would materialise dres = d(bn3)/d(residual), then add it to conv1's
    dX in a separate elementwise pass (read 2 tensors, write 1) before the previous block's BN
    backward reads the sum twice. With a link (created by the previous block for y):
      * the block's bn3 backward parks dres here and returns no gradient for the residual;
      * either conv1's backward GEMM accumulates into it (``models.resnet._Conv1x1Fn``, beta = 1),
      * or the previous block's BN backward reads it as a second output gradient ``dy2`` and
        sums it on load (``bn_bwd`` with dy2) — the add pass disappears.
    bn3's backward always runs before conv1's and before the previous block's BN backward (both
    depend on it through the graph), so the hand-off is ordered by the graph itself."""
    __slots__ = ("grad", "closed", "bn_ctx", "sums")

    def __init__(self):
        self.grad = None
        self.closed = False
        # set by a producer tail that applies its BN backward inside its convs (ops.conv
        # bnrelu_conv1x1_bn_res): (z, mask, mean, invstd) of that BN, so the consumer's conv1
        # data-gradient kernel can also emit the BN's backward sums -> sums = (sdz, sdzx, ptr)
        self.bn_ctx = None
        self.sums = None

    def take(self):
        """Consumer side: the parked gradient (a tensor, a ``MaskedGrad`` or None); later
        producers keep their own."""
        g, self.grad = self.grad, None
        self.closed = True
        return g

    def take_tensor(self):
        """``take`` with a ``MaskedGrad`` / ``ops.conv.S2Grad`` materialised (consumers without the
        matching epilogue)."""
        g = self.take()
        return g.materialize() if hasattr(g, "materialize") else g


class MaskedGrad:
    """A residual gradient m * g left unmaterialised: g is the block-output gradient (NHWC bf16)
    and m the forward's ReLU bit mask ([M, C/8] bytes, bit k of byte j = channel 8 j + k). The
    1x1 data-gradient kernel adds it in its epilogue (``lib().conv1x1_link``); anything else calls
    ``materialize``."""
    __slots__ = ("g", "mask")

    def __init__(self, g: torch.Tensor, mask: torch.Tensor):
        self.g = g
        self.mask = mask

    def materialize(self) -> torch.Tensor:
        g = self.g
        N, C, H, W = g.shape
        shifts = torch.arange(8, device=g.device, dtype=torch.uint8)
        bits = (self.mask.view(-1, C // 8, 1) >> shifts) & 1
        rows = g.permute(0, 2, 3, 1).reshape(-1, C) * bits.view(-1, C).to(g.dtype)
        return rows.view(N, H, W, C).permute(0, 3, 1, 2)


# how often link_tap parked its gradient vs fell back to a normal add (tests pin the order)
TAP_STATS = {"parked": 0, "fallback": 0}


class _LinkTapFn(torch.autograd.Function):
    """Identity whose backward parks the incoming gradient on a ResidualLink instead of
    returning it, so a GEMM consumer on a parallel branch can absorb it with its beta = 1
    epilogue (a downsample block's input feeds both down_conv and conv1: their two data
    gradients would otherwise meet in an elementwise add). If the consumer already ran, the
    gradient flows normally and autograd adds it."""

    @staticmethod
    def forward(ctx, x, link):
        ctx.link = link
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        link = ctx.link
        if link.closed or link.grad is not None:
            TAP_STATS["fallback"] += 1
            return g, None
        TAP_STATS["parked"] += 1
        link.grad = g.contiguous(memory_format=torch.channels_last) if g.dim() == 4 else g.contiguous()
        return None, None


def link_tap(x: torch.Tensor, link: "ResidualLink") -> torch.Tensor:
    return _LinkTapFn.apply(x, link)


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, res, rmean, rvar, mean_in, invstd_in, eps, momentum, relu,
                training, res_link, out_link):
        has_res = res is not None
        want_mask = has_res and relu and any(ctx.needs_input_grad[:4])
        y, mean, invstd, mask = lib().bn_fwd(x, res, gamma, beta, rmean, rvar, mean_in,
                                             invstd_in, eps, momentum, relu, training, want_mask)
        # the residual itself is never needed again: its ReLU contribution lives in the bit mask
        ctx.save_for_backward(x, mask if want_mask else None, gamma, beta, mean, invstd)
        ctx.relu = relu
        ctx.has_res = has_res
        ctx.res_link = res_link
        ctx.out_link = out_link
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, gamma, beta, mean, invstd = ctx.saved_tensors
        dy2 = ctx.out_link.take_tensor() if ctx.out_link is not None else None
        dx, dg, db, dres = lib().bn_bwd(dy, dy2, x, mask, gamma, beta, mean, invstd, ctx.relu,
                                        ctx.has_res)
        if ctx.has_res and ctx.res_link is not None:
            ctx.res_link.grad = dres
            dres = None
        return (dx, dg, db, dres if ctx.has_res else None, None, None, None, None, None, None,
                None, None, None, None)


class _BNAddBNActFn(torch.autograd.Function):
    """y = relu(bn_a(x1) + bn_b(x2)) for a downsample block's tail (bn3 of the main branch plus
    the shortcut BN) without materialising the shortcut BN's output or its gradient."""

    @staticmethod
    def forward(ctx, x1, g1, b1, x2, g2, b2, rm1, rv1, rm2, rv2, stats_in, eps, momentum,
                training, out_link):
        want_mask = any(ctx.needs_input_grad[:6])
        m1 = i1 = m2 = i2 = None
        if not training:
            m1, i1, m2, i2 = stats_in
        y, m1, i1, m2, i2, mask = lib().bn_fwd2(x1, x2, g1, b1, g2, b2, rm1, rv1, rm2, rv2, m1,
                                                i1, m2, i2, eps, momentum, training, want_mask)
        ctx.save_for_backward(x1, x2, mask if want_mask else None, g1, g2, m1, i1, m2, i2)
        ctx.out_link = out_link
        return y

    @staticmethod
    def backward(ctx, dy):
        x1, x2, mask, g1, g2, m1, i1, m2, i2 = ctx.saved_tensors
        dy2 = ctx.out_link.take_tensor() if ctx.out_link is not None else None
        dx1, dg1, db1, dx2, dg2, db2 = lib().bn_bwd2(dy, dy2, x1, x2, mask, g1, g2, m1, i1, m2, i2)
        return (dx1, dg1, db1, dx2, dg2, db2) + (None,) * 9


def bn_add_bn_relu(x1: torch.Tensor, bn1: "BatchNormAct2d", x2: torch.Tensor,
                   bn2: "BatchNormAct2d", out_link: Optional[ResidualLink] = None,
                   stats: Optional[tuple] = None) -> torch.Tensor:
    """relu(bn1(x1) + bn2(x2)) with bn1 / bn2 training-mode BatchNorms (bn1.relu applies to the
    sum, bn2 has no ReLU). Fused path: bf16 channels_last GPU tensors of equal shape. ``stats`` =
    (mean1, invstd1, mean2, invstd2): batch statistics already computed by the producing convs
    (training only; running statistics already updated)."""
    if (_fused_ok(x1, bn1.weight) and _fused_ok(x2, bn2.weight) and x1.shape == x2.shape
            and not bn2.relu and bn1.relu and bn1.eps == bn2.eps and bn1.momentum == bn2.momentum):
        if stats is not None and bn1.training:
            return _BNAddBNActFn.apply(x1, bn1.weight, bn1.bias, x2, bn2.weight, bn2.bias, None,
                                       None, None, None, tuple(stats), bn1.eps, bn1.momentum,
                                       False, out_link)
        stats = None
        if not bn1.training:
            stats = (bn1.running_mean.float(), torch.rsqrt(bn1.running_var.float() + bn1.eps),
                     bn2.running_mean.float(), torch.rsqrt(bn2.running_var.float() + bn2.eps))
        return _BNAddBNActFn.apply(x1, bn1.weight, bn1.bias, x2, bn2.weight, bn2.bias,
                                   bn1.running_mean if bn1.training else None,
                                   bn1.running_var if bn1.training else None,
                                   bn2.running_mean if bn2.training else None,
                                   bn2.running_var if bn2.training else None, stats, bn1.eps,
                                   bn1.momentum, bn1.training, out_link)
    return bn1(x1, residual=bn2(x2), out_link=out_link)


def fused_ok(x: torch.Tensor, gamma: torch.Tensor) -> bool:
    return _fused_ok(x, gamma)


def _fused_ok(x: torch.Tensor, gamma: torch.Tensor) -> bool:
    if not (x.is_cuda and x.dtype == torch.bfloat16 and gamma.dtype == torch.bfloat16):
        return False
    if not _P().fused_bn:     # PerfPolicy.library(): PyTorch's BatchNorm composition
        return False
    C = x.shape[1]
    if C % 8 or C > 2048 or 256 % (C // 8):
        return False
    return x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)


def bn_act(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor,
           running_mean: Optional[torch.Tensor], running_var: Optional[torch.Tensor],
           residual: Optional[torch.Tensor] = None, relu: bool = True, training: bool = True,
           momentum: float = 0.1, eps: float = 1e-5,
           res_link: Optional[ResidualLink] = None,
           out_link: Optional[ResidualLink] = None,
           stats: Optional[tuple] = None) -> torch.Tensor:
    """``res_link`` / ``out_link``: see ResidualLink; only honoured on the fused path (callers
    check ``fused_ok`` before creating links). ``stats`` = (mean, invstd): the training batch
    statistics of x, already computed by its producer (``ops.conv``: the conv epilogue, which also
    updated the running statistics) — only the apply pass runs."""
    if _fused_ok(x, gamma) and (residual is None or residual.is_contiguous(
            memory_format=torch.channels_last)):
        if training and stats is not None:
            return _BNActFn.apply(x, gamma, beta, residual, None, None, stats[0], stats[1], eps,
                                  momentum, relu, False, res_link, out_link)
        if training:
            return _BNActFn.apply(x, gamma, beta, residual, running_mean, running_var, None, None,
                                  eps, momentum, relu, True, res_link, out_link)
        invstd = torch.rsqrt(running_var.float() + eps)
        return _BNActFn.apply(x, gamma, beta, residual, None, None, running_mean.float(), invstd,
                              eps, momentum, relu, False, res_link, out_link)
    # reference composition (CPU / unsupported layouts)
    y = F.batch_norm(x, running_mean, running_var, gamma, beta, training, momentum, eps) \
        if running_mean is None or running_mean.dtype == x.dtype else \
        _bn_mixed(x, gamma, beta, running_mean, running_var, training, momentum, eps)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


def _bn_mixed(x, gamma, beta, rm, rv, training, momentum, eps):
    """F.batch_norm with fp32 running stats and lower-precision activations."""
    xf = x.float()
    y = F.batch_norm(xf, rm, rv, gamma.float(), beta.float(), training, momentum, eps)
    return y.to(x.dtype)


class BatchNormAct2d(nn.Module):
    def __init__(self, num_features: int, relu: bool = True, eps: float = 1e-5,
                 momentum: float = 0.1):
        super().__init__()
        self.num_features = num_features
        self.relu = relu
        self.eps = eps
        self.momentum = momentum
        self.weight = nn.Parameter(torch.ones(num_features))
        self.bias = nn.Parameter(torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))

    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        # keep running statistics in fp32 whatever dtype the module is cast to
        for k in ("running_mean", "running_var"):
            b = self._buffers[k]
            if b is not None and b.dtype != torch.float32:
                self._buffers[k] = b.float()
        return self

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                res_link: Optional[ResidualLink] = None,
                out_link: Optional[ResidualLink] = None,
                stats: Optional[tuple] = None) -> torch.Tensor:
        return bn_act(x, self.weight, self.bias, self.running_mean, self.running_var, residual,
                      self.relu, self.training, self.momentum, self.eps, res_link, out_link,
                      stats)

    def extra_repr(self) -> str:
        return f"{self.num_features}, relu={self.relu}"
