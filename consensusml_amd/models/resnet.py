"""ResNet-50 (He et al. 2016, v1.5: stride on the 3x3 conv) for the headline benchmark (N12).

Convolutions run on MIOpen in bf16 with channels_last activations and weights (NHWC is MIOpen's
fast layout on CDNA). Every BatchNorm is a ``BatchNormAct2d``: BN + (residual add) + ReLU fused
into the HIP kernels of ``csrc/kernels/bn_act.hip`` on GPU — the block tail
``relu(bn3(conv3(x)) + identity)`` is one op. Random-init weights (no checkpoints offline).
BASELINE.json config: "ResNet-50 bf16 DP=8 with Krum".
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import conv as fconv
from ..ops.bn import BatchNormAct2d, ResidualLink, bn_add_bn_relu, fused_ok, link_tap
from ..ops.pool import bn_relu_max_pool2d, max_pool2d
from ..ops.stem import stem_conv_bn_relu_pool, stem_ok

# Every kernel / fusion choice of this model is a field of the typed PerfPolicy
# (consensusml_amd.perf), read when the model runs: ``perf.use_policy(...)`` switches paths inside
# one process, and benchmark lines / checkpoints record the policy in force.
from ..perf import policy as _P


def recompute_tail_policy(planes: int) -> bool:
    """Measured at batch 2048 (profiles/r02_recompute_tail35/): up to 128 planes 152.1 -> 145.2
    ms / step; adding layer 3 (256) another -1.1 ms; layer 4 (512) +0.4-0.6 ms back."""
    p = _P()
    return (p.recompute_tail and planes <= p.recompute_tail_max_planes
            and fconv.recompute_tail_ok(planes))


def fused_bn3_bwd_policy(planes: int) -> bool:
    """Whether an identity block uses the fused tail backward. Measured per stage at batch 2048
    (bench/bwd_fusion.py, profiles/r02_bwd_fusion15.jsonl): layers 1-2 are bandwidth-bound and
    gain 1.28 / 0.34 ms per block; on layers 3-4 (14 x 14, 7 x 7) the library GEMMs the fusion
    replaces are faster than the fused kernels (-0.31 / -0.73 ms per block; -0.12 / -0.51 with
    the MT = 2 tiles, profiles/r02_19_mt2/r02_19_bwdfusion.jsonl)."""
    from ..ops import conv as _c
    p = _P()
    return p.fused_bn3_bwd and planes <= p.fused_bn3_bwd_max_planes and _c.res_tail_ok(planes)


def fused_conv1x1_policy(cin: int, cout: int, hw_out: int, stride: int, prologue: bool) -> bool:
    """Whether a 1x1 conv + BN runs as the fused kernel. Measured per shape at batch 2048
    (bench/conv1x1_fused.py, profiles/r02_conv1x1_04.jsonl): the fused kernel streams x / y at
    ~5 TB/s, so it wins wherever the conv is memory-bound (28 x 28 and larger outputs: 0.07-0.83
    ms saved per call) and whenever it also removes bn2's apply pass (every conv3); on the
    14 x 14 / 7 x 7 shapes with 1024+ input channels the library GEMMs (0.7-1 PFLOP/s) beat it
    by more than the statistics pass it saves (0.03-0.14 ms)."""
    if not _P().fused_conv1x1:
        return False
    if prologue:
        return True
    return hw_out >= 784


def conv1x1_policy(cin: int, cout: int, hw: int):
    """(forward as GEMM, data gradient as GEMM) for a 1x1 stride-1 conv."""
    mode = _P().conv1x1_gemm
    if mode is True or mode == "gemm":
        return True, True
    if mode is False or mode == "miopen":
        return False, False
    # PerfPolicy.c1_dgrad64_gemm: layer 1.0's 64 -> 64 conv1 data gradient as a GEMM too, so the
    # downsample's dX is absorbed by its beta = 1 epilogue (one pass) instead of MIOpen's data
    # gradient plus the stem pool backward's two-gradient sum (pool_gsum): -0.4 ms/step at batch
    # 2560 (profiles/r06_30/)
    if cin == 64 and cout == 64 and _P().c1_dgrad64_gemm:
        return False, True
    return cin >= 1024, (cout < cin) or hw <= 196


class _Conv1x1Fn(torch.autograd.Function):
    """1x1 stride-1 conv on a channels_last tensor x [N, C, H, W] (= row-major [M, C] rows).

    forward: y = x W^T as one GEMM (fwd_gemm) or MIOpen. backward: dX = dY W as a GEMM
    (dgrad_gemm; accumulated in place into a residual gradient parked on ``link`` — the GEMM's
    beta = 1 epilogue replaces an elementwise add) or MIOpen; dW from ``csrc/kernels/wgrad1x1.hip``
    (own_wgrad: split-K MFMA over the pixels, both operands through transposed LDS reads) or
    MIOpen's backward-weight (``aten.convolution_backward`` with only the weight output)."""

    @staticmethod
    def forward(ctx, x, w, link, fwd_gemm, dgrad_gemm, own_wgrad=False):
        ctx.save_for_backward(x, w)
        ctx.link = link
        ctx.wt = fconv.cached_wt(w)   # W^T from the forward's layout prefetch, if any
        ctx.dgrad_gemm = dgrad_gemm
        ctx.own_wgrad = own_wgrad
        N, C, H, W = x.shape
        if fwd_gemm:
            y = fconv.conv_mm(x.permute(0, 2, 3, 1).reshape(N * H * W, C), w.reshape(w.shape[0], C))
            return y.view(N, H, W, w.shape[0]).permute(0, 3, 1, 2)
        return F.conv2d(x, w)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        N, C, H, W = x.shape
        Co = w.shape[0]
        need_dx = ctx.needs_input_grad[0]
        mio_dx = need_dx and not ctx.dgrad_gemm
        own_dw = ctx.own_wgrad and ctx.needs_input_grad[1]
        mio_dw = ctx.needs_input_grad[1] and not own_dw
        dx_m, dw, h = None, None, None
        if own_dw:   # on the side stream (large batches) while the data gradient runs
            from ..ops.native import lib
            dw, h = fconv._wgrad_fork(lambda d, a, b: lib().wgrad1x1(d, a, b.dtype).view_as(b),
                                      dy, x, w, conv1x1=True)
        if mio_dx or mio_dw:
            dx_m, dw_m, _ = torch.ops.aten.convolution_backward(
                dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                [mio_dx, mio_dw, False])
            if mio_dw:
                dw = dw_m
        dx = dx_m if mio_dx else None
        if need_dx and ctx.dgrad_gemm:
            dy2 = dy.permute(0, 2, 3, 1).reshape(N * H * W, Co)
            w2 = w.reshape(Co, C)
            link = ctx.link
            g = link.take() if link is not None else None
            if isinstance(g, fconv.MaskedGrad):
                dx = fconv.masked_link_dgrad(dy, w, g, link, ctx.wt)
                return dx, fconv._wgrad_join(dw, h), None, None, None, None
            if isinstance(g, fconv.S2Grad):
                g = g.materialize()
            w_nk = fconv.dgrad_wnk(dy2, w2, ctx.wt)
            if g is not None:
                dres = g.permute(0, 2, 3, 1).reshape(N * H * W, C) if g.dim() == 4 else g
                if dres.data_ptr() == g.data_ptr() and dres.is_contiguous():
                    d2 = fconv.conv_mm(dy2, w_nk, acc=dres)   # beta = 1 epilogue, in place
                else:
                    d2 = torch.addmm(dres, dy2, w2)
            else:
                d2 = fconv.conv_mm(dy2, w_nk)
            dx = d2.view(N, H, W, C).permute(0, 3, 1, 2)
        return dx, fconv._wgrad_join(dw, h), None, None, None, None


# (cin, cout) of the stride-1 1x1 convs whose weight gradient runs on wgrad1x1.hip. In isolation the
# kernel beats MIOpen on all nine >= 128-channel shapes at batch 1024 (tools/diag/wgrad1x1_bench.py,
# profiles/r01_wgrad1x1_60.txt); in the training step the five with the largest margins are the best
# set: 12,011 img/s vs 11,991 for all nine and 11,929-11,958 for none (profiles/r01_bench62_*.json,
# same box). The 64-channel layer-1 shapes are at the HBM floor on MIOpen.
_CORE = {(128, 512), (512, 128), (256, 1024), (512, 2048), (2048, 512)}
_ALL = _CORE | {(256, 128), (512, 256), (1024, 256), (1024, 512)}
# + the layer-4 downsample (its input pre-subsampled to 7 x 7, so a stride-1 1x1)
_WIDE = _ALL | {(1024, 2048)}
_SETS = {"core": _CORE, "all": _ALL, "wide": _WIDE}


def own_wgrad_ok(cin: int, cout: int) -> bool:
    p = _P()
    return p.own_wgrad1x1 and (cin, cout) in _SETS[p.wgrad1x1_set]


class Conv1x1(nn.Conv2d):
    """1x1 convolution. With stride 1 on a channels_last GPU tensor the NHWC activation IS a
    row-major [N*H*W, C] matrix, so the forward and the data gradient can be single GEMMs (no
    im2col, no layout change) — chosen per shape by ``conv1x1_policy``. Strided 1x1 (downsample)
    convs and CPU tensors use the regular MIOpen / ATen convolution. Same parameter as
    nn.Conv2d."""

    def __init__(self, cin: int, cout: int, stride: int = 1):
        super().__init__(cin, cout, 1, stride=stride, bias=False)

    def _policy(self, x: torch.Tensor):
        if not (self.stride == (1, 1) and x.is_cuda and x.dim() == 4
                and x.is_contiguous(memory_format=torch.channels_last)):
            return False, False
        return conv1x1_policy(self.in_channels, self.out_channels, x.shape[2] * x.shape[3])

    def link_ok(self, x: torch.Tensor) -> bool:
        """True when the data gradient is a GEMM that can absorb a parked residual gradient."""
        return self._policy(x)[1]

    def forward(self, x: torch.Tensor, res_link: Optional[ResidualLink] = None) -> torch.Tensor:
        fwd_gemm, dgrad_gemm = self._policy(x)
        own = (self.stride == (1, 1) and x.is_cuda and x.dtype == torch.bfloat16
               and self.weight.dtype in (torch.bfloat16, torch.float32)
               and x.is_contiguous(memory_format=torch.channels_last)
               and own_wgrad_ok(self.in_channels, self.out_channels))
        if fwd_gemm or dgrad_gemm or own:
            return _Conv1x1Fn.apply(x, self.weight, res_link if dgrad_gemm else None, fwd_gemm,
                                    dgrad_gemm, own)
        return super().forward(x)


class _GlobalAvgPoolFn(torch.autograd.Function):
    """[N, C, H, W] channels_last -> [N, C]. ATen's adaptive_avg_pool2d backward hands the next
    BN backward a gradient that is then re-laid out to NHWC by a strided copy (0.63 ms per
    batch-2048 step, ``profiles/r01_copies2048.txt``); here the broadcast of dy / (H W) is
    written straight into NHWC memory (one write-only pass, 0.14 ms). Same fp32 divide, same rounding."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)

    @staticmethod
    def backward(ctx, g):
        N, C, H, W = ctx.shape
        if g.is_cuda and g.dtype == torch.bfloat16 and C % 8 == 0:
            from ..ops.native import lib   # one launch (was a divide, a cast and a cat)
            return lib().avgpool_bwd(g, H, W)
        gs = (g.float() / (H * W)).to(g.dtype).contiguous()
        # a concatenation of H W copies writes at 2.8 TB/s, a broadcast copy_ at 1.6
        # (tools/diag/avgpool_bwd_bench.py)
        return torch.cat([gs] * (H * W), dim=1).view(N, H, W, C).permute(0, 3, 1, 2)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    if _P().nhwc_avgpool and x.is_cuda and x.dim() == 4 \
            and x.is_contiguous(memory_format=torch.channels_last):
        return _GlobalAvgPoolFn.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)


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

    def _conv2(self, x: torch.Tensor) -> torch.Tensor:
        if _P().own_dgrad3x3 and self.training:
            return fconv.conv3x3(x, self.conv2)
        return self.conv2(x)

    def _down_s2_compact_ok(self, x: torch.Tensor, dlink) -> bool:
        c = self.down_conv
        return (dlink is not None and _P().down_s2_compact and c.stride == (2, 2)
                and x.is_cuda and x.dtype == torch.bfloat16 and x.shape[1] % 8 == 0
                and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0
                and x.is_contiguous(memory_format=torch.channels_last))

    def _down_conv_s2_compact(self, x: torch.Tensor, dlink) -> torch.Tensor:
        """The stride-2 downsample conv as a stride-1 1x1 conv of x[:, :, ::2, ::2] (one subsample
        pass): forward / data gradient as plain GEMMs at the compact resolution, and the compact
        data gradient parked on conv1's link (``subsample2_link``) for conv1's data-gradient GEMM to
        take -- instead of MIOpen's stride-2 backward-data, which zero-fills and writes a
        full-resolution gradient (layer 4: 1024 -> 2048 at 14 x 14 -> 7 x 7)."""
        c = self.down_conv
        xs = fconv.subsample2_link(x, dlink)
        fwd, dg = conv1x1_policy(c.in_channels, c.out_channels, xs.shape[2] * xs.shape[3])
        return _Conv1x1Fn.apply(xs, c.weight, None, fwd, dg,
                                own_wgrad_ok(c.in_channels, c.out_channels))

    def _fused_ok(self, x: torch.Tensor) -> bool:
        return (_P().fused_conv1x1 and self.training and torch.is_grad_enabled()
                and fconv.fused_conv_ok(x, self.conv1.weight)
                and fused_ok(x, self.bn3.weight))

    def _conv_bn(self, x, conv: "Conv1x1", bn, link=None):
        """(z, stats) of a 1x1 conv followed by a BN: fused kernel when the policy picks it, else
        the library conv (stats None: the BN computes them)."""
        st = conv.stride[0]
        hw = (x.shape[2] // st) * (x.shape[3] // st)
        if fused_conv1x1_policy(conv.in_channels, conv.out_channels, hw, st, False):
            dg = st == 1 and conv1x1_policy(conv.in_channels, conv.out_channels, hw)[1]
            # stride 2: ops.conv._wgrad takes the stride-2 DMA kernel's single-tap form
            own = own_wgrad_ok(conv.in_channels, conv.out_channels) if st == 1 else True
            z, m, i = fconv.conv1x1_bn_stats(x, conv, bn, st, dg, own, link if dg else None)
            return z, (m, i)
        if st == 1:
            return conv(x, res_link=link if conv.link_ok(x) else None), None
        return conv(x), None

    def _forward_fused(self, x: torch.Tensor, use_links: bool) -> torch.Tensor:
        """Training forward with the fused conv + BN kernels (ops.conv): bn1 / bn3 / down_bn get
        their statistics from the conv epilogues, bn2 + ReLU is applied inside conv3."""
        if self.down_conv is None:
            link = getattr(x, "_cml_link", None) if use_links else None
            z1, st1 = self._conv_bn(x, self.conv1, self.bn1, link)
            dlink = None
        else:
            link = None
            dlink = ResidualLink() if use_links and self.conv1.link_ok(x) else None
            z1, st1 = self._conv_bn(x, self.conv1, self.bn1, dlink)
        planes = self.conv3.in_channels
        hw2 = (z1.shape[2] // self.conv2.stride[0]) * (z1.shape[3] // self.conv2.stride[0])
        fuse3 = fused_conv1x1_policy(planes, planes * 4, hw2, 1, True)
        pol = _P()
        own3 = (fuse3 and pol.conv3x3_bn_stats and pol.own_dgrad3x3
                and fconv.conv3x3_ok(z1, self.conv2))
        if (own3 and pol.bn1_dgrad_sums and st1 is None and pol.bn1_sums_lib_conv1
                and self.bn1.training and fused_ok(z1, self.bn1.weight)):
            # conv1 ran on the library (layers 3-4, 14 x 14 / 7 x 7): one statistics pass here
            # (the module BN would make the same one), so that bn1's backward also takes its sums
            # from the 3x3 data gradient's epilogue instead of a reduction pass over dy1 and z1
            st1 = fconv.bn_stats(z1, self.bn1)
        own3s2 = (fuse3 and not own3 and pol.own_conv3x3_s2
                  and fconv.conv3x3_s2_ok(z1, self.conv2))
        if own3 and pol.bn1_dgrad_sums and st1 is not None and self.bn1.training:
            # bn1's backward sums come from the 3x3 data gradient's epilogue
            z2, st2 = fconv.bnrelu_conv3x3_bn_stats(z1, self.bn1, st1, self.conv2, self.bn2)
        elif (own3s2 and pol.bn1_dgrad_sums and st1 is not None and self.bn1.training
                and fused_ok(z1, self.bn1.weight)):
            # stride-2 conv of a downsample block: the same, with the parity-class data gradient
            z2, st2 = fconv.bnrelu_conv3x3_s2_bn_stats(z1, self.bn1, st1, self.conv2, self.bn2)
        elif own3s2:
            z2, st2 = fconv.conv3x3_s2_bn_stats(self.bn1(z1, stats=st1), self.conv2, self.bn2)
        else:
            out = self.bn1(z1, stats=st1)
            if own3:
                z2, st2 = fconv.conv3x3_bn_stats(out, self.conv2, self.bn2)
            else:
                z2 = self._conv2(out)
                st2 = fconv.bn_stats(z2, self.bn2) if fuse3 else None
        if fuse3:
            rec = self.down_conv is None and recompute_tail_policy(planes)
            if rec or (self.down_conv is None and fused_bn3_bwd_policy(planes)):
                out_link = ResidualLink() if use_links else None
                tail = fconv.bnrelu_conv1x1_bn_res_recompute if rec \
                    else fconv.bnrelu_conv1x1_bn_res
                y = tail(z2, self.bn2, st2, self.conv3, self.bn3, x, link, out_link)
                if out_link is not None:
                    y._cml_link = out_link
                return y
            if (self.down_conv is not None and pol.recompute_down_tail and self.bn3.eps ==
                    self.down_bn.eps and fconv.down_tail_recompute_s2_ok(x, planes, self.down_conv)):
                # stride-2 downsample tail: the stride-1 recompute kernels on x[:, :, ::2, ::2];
                # its gradient (zero-filled full resolution) parks on conv1's link as before
                out_link = ResidualLink() if use_links else None
                y = fconv.down_tail_recompute(z2, self.bn2, st2, self.conv3, self.bn3,
                                              fconv.subsample2_link(x, dlink), self.down_conv,
                                              self.down_bn, out_link)
                if out_link is not None:
                    y._cml_link = out_link
                return y
            if (self.down_conv is not None and pol.recompute_down_tail and self.bn3.eps ==
                    self.down_bn.eps and fconv.down_tail_recompute_ok(x, planes, self.down_conv)):
                out_link = ResidualLink() if use_links else None
                tlink = dlink if dlink is not None else \
                    (getattr(x, "_cml_pool_link", None) if use_links else None)
                xin = link_tap(x, tlink) if tlink is not None else x
                y = fconv.down_tail_recompute(z2, self.bn2, st2, self.conv3, self.bn3, xin,
                                              self.down_conv, self.down_bn, out_link)
                if out_link is not None:
                    y._cml_link = out_link
                return y
            dg = conv1x1_policy(planes, planes * 4, hw2)[1]
            z, m3, i3 = fconv.bnrelu_conv1x1_bn_stats(z2, self.bn2, st2, self.conv3, self.bn3, dg,
                                                      own_wgrad_ok(planes, planes * 4)
                                                      or planes == 64)
            st3 = (m3, i3)
        else:
            z, st3 = self.conv3(self.bn2(z2)), None
        out_link = ResidualLink() if use_links else None
        if self.down_conv is None:
            y = self.bn3(z, residual=x, res_link=link, out_link=out_link, stats=st3)
        else:
            tlink = dlink if dlink is not None else \
                (getattr(x, "_cml_pool_link", None) if use_links else None)
            if self._down_s2_compact_ok(x, dlink):
                zd, std = self._down_conv_s2_compact(x, dlink), None
            else:
                xin = link_tap(x, tlink) if tlink is not None else x
                zd, std = self._conv_bn(xin, self.down_conv, self.down_bn)
            stats = None if (st3 is None or std is None) else st3 + std
            if stats is None and (st3 is not None or std is not None):
                # one side fused, the other not: let the unfused side compute its statistics
                y = self.bn3(z, residual=self.down_bn(zd, stats=std), out_link=out_link,
                             stats=st3)
            else:
                y = bn_add_bn_relu(z, self.bn3, zd, self.down_bn, out_link, stats=stats)
        if out_link is not None:
            y._cml_link = out_link
        return y

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        use_links = _P().residual_link and torch.is_grad_enabled() and self.training
        if self._fused_ok(x):
            return self._forward_fused(x, use_links)
        if self.down_conv is None:
            # identity block: bn3's residual gradient is parked on the link of our input (made by
            # the producing block); conv1's GEMM backward (if used) or the producer's BN backward
            # consumes it (see ops.bn.ResidualLink)
            link = getattr(x, "_cml_link", None) if use_links else None
            out = self.bn1(self.conv1(x, res_link=link if self.conv1.link_ok(x) else None))
            out = self.bn2(self._conv2(out))
            z = self.conv3(out)
            fused = fused_ok(z, self.bn3.weight)
            out_link = ResidualLink() if use_links and fused else None
            y = self.bn3(z, residual=x, res_link=link if fused else None, out_link=out_link)
        else:
            # x feeds conv1 and down_conv. When conv1's data gradient is a GEMM, down_conv's dX is
            # parked on a link (link_tap) and absorbed by that GEMM's beta = 1 epilogue instead of
            # an elementwise add. The downsample branch is built after the main branch so that
            # autograd (ready nodes in reverse creation order) runs its backward first; the link
            # falls back to a normal add if that order ever changes.
            dlink = ResidualLink() if use_links and self.conv1.link_ok(x) else None
            # otherwise, when x is the fused stem's output, its pool backward takes the parked
            # gradient as a second input (ops.stem._StemFn)
            tlink = dlink if dlink is not None else \
                (getattr(x, "_cml_pool_link", None) if use_links else None)
            out = self.bn1(self.conv1(x, res_link=dlink))
            out = self.bn2(self._conv2(out))
            z = self.conv3(out)
            zd = self.down_conv(link_tap(x, tlink) if tlink is not None else x)
            out_link = ResidualLink() if use_links and fused_ok(z, self.bn3.weight) else None
            # relu(bn3(z) + down_bn(zd)) in one op: the shortcut BN output is never stored
            y = bn_add_bn_relu(z, self.bn3, zd, self.down_bn, out_link) if _P().fuse_down_bn \
                else self.bn3(z, residual=self.down_bn(zd), out_link=out_link)
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

    def stem(self, x: torch.Tensor) -> torch.Tensor:
        """7x7/2 conv. bf16 NHWC GPU images with 3 channels are zero-padded to 4 (one HIP pass)
        and the weight likewise (a view-sized pad), so MIOpen runs its vectorised NHWC kernels:
        1.4x faster forward and weight gradient (bench/stem_pad.py). Same math, same parameter."""
        w = self.conv1.weight
        if (_P().stem_pad4 and x.is_cuda and x.dtype == torch.bfloat16 and x.shape[1] == 3
                and x.is_contiguous(memory_format=torch.channels_last) and not x.requires_grad):
            from ..ops.native import lib
            x4 = lib().pad_c4(x)
            w4 = F.pad(w, (0, 0, 0, 0, 0, 1)).contiguous(memory_format=torch.channels_last)
            return F.conv2d(x4, w4, stride=2, padding=3)
        return self.conv1(x)

    def _make(self, planes: int, blocks: int, stride: int) -> nn.Sequential:
        down = stride != 1 or self.inplanes != planes * 4
        mods = [Bottleneck(self.inplanes, planes, stride, down)]
        self.inplanes = planes * 4
        mods += [Bottleneck(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*mods)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        pol = _P()
        if pol.fuse_stem_conv and stem_ok(x, self.conv1, self.bn1):
            plink = ResidualLink() if (pol.pool_link and pol.residual_link and self.training
                                       and torch.is_grad_enabled()) else None
            x = stem_conv_bn_relu_pool(x, self.conv1, self.bn1, plink)
            if plink is not None:
                x._cml_pool_link = plink    # layer1.0's downsample conv parks its dX here
        elif pol.fuse_stem_pool:
            x = bn_relu_max_pool2d(self.stem(x), self.bn1, 3, 2, 1)
        else:
            x = max_pool2d(self.bn1(self.stem(x)), 3, 2, 1)
        # every block's 3x3 weight layouts (implicit-GEMM forward / data gradient) and conv1
        # transpose (1x1 data-gradient operand) in one launch for this forward
        # (PerfPolicy.batch_wlayouts) instead of one per conv
        blocks = [b for layer in (self.layer1, self.layer2, self.layer3, self.layer4)
                  for b in layer]
        batched = (pol.batch_wlayouts and self.training and torch.is_grad_enabled()
                   and fconv.prefetch_wlayouts([b.conv2.weight for b in blocks]
                                               + [b.conv1.weight for b in blocks]))
        try:
            x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        finally:
            if batched:
                fconv.clear_wlayouts()
        return self.fc(global_avg_pool(x))


def resnet50(num_classes: int = 1000) -> ResNet:
    return ResNet([3, 4, 6, 3], num_classes)


def resnet_tiny(num_classes: int = 10) -> ResNet:
    """Same block structure at width 8 / one block per stage (tests)."""
    return ResNet([1, 1, 1, 1], num_classes, width=8)
