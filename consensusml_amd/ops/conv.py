"""1x1 convolutions fused with the BatchNorm around them (``csrc/kernels/conv1x1.hip``).

A ResNet bottleneck is conv1 (1x1) -> bn1 + ReLU -> conv2 (3x3) -> bn2 + ReLU -> conv3 (1x1) ->
bn3 (+ residual) + ReLU. Unfused, every training BN first re-reads its input for the batch
statistics, and bn2's output y2 is written only to be read back by conv3. Here:

* ``conv1x1_bn_stats``: the 1x1 conv (stride 1 or 2) emits the BN statistics of its output from
  the MFMA accumulators (its BN then runs only the apply pass);
* ``bnrelu_conv1x1_bn_stats``: conv3 reads bn2's *input* z2 and applies bn2 + ReLU while staging
  its operand (y2 is never written or read), and emits bn3's statistics. Its backward recomputes
  y2 on the fly inside the MFMA weight-gradient kernel (``wgrad1x1.hip`` prologue) and runs bn2's
  backward on the data gradient.

The statistics are the exact batch statistics of the bf16 conv output (sums of the rounded
values, shifted by the running mean, folded in fp64), so the BatchNorm forward and backward are
the ordinary training ones; running statistics are updated by the finalize kernel.
Gradients: data gradient as a hipBLASLt GEMM (stride 1, per-shape policy of
``models.resnet.conv1x1_policy``) or MIOpen; weight gradient on ``wgrad1x1.hip`` or MIOpen.

* ``bnrelu_conv1x1_bn_res``: the identity-block tail, whose backward never materialises bn3's
  input gradient or the residual gradient (bn3's backward runs inside conv3's gradient kernels and
  the next conv1 data-gradient epilogue; see _BNReLUConv1x1BNResFn and ``masked_link_dgrad``).
"""
from __future__ import annotations

from typing import Optional, Tuple, Dict

import torch
import torch.nn.functional as F

from ..perf import policy as _P
from .bn import MaskedGrad
from .native import lib


def fused_conv_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Shapes / layouts the fused kernel takes (else callers use the unfused path)."""
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last) and x.shape[1] % 64 == 0
            and w.shape[0] % 64 == 0 and w.shape[2] == 1 and w.shape[3] == 1)


def _nt_tile(a: torch.Tensor, M: int, N: int, K: int) -> int:
    """Tile of the gemm.hip kernel that takes this 1x1-conv GEMM, or 0 (hipBLASLt): policy on,
    bf16 GPU operands, then ``gemm_nt_pick`` -- the 256 x 256 kernel once it has >= 128 tiles
    (it fills the chip), else the 128 x 128 one (the layer-4 GEMMs of a batch-256 rank: 34.9-37.0
    vs 43.2-44.6 us on the 256 tile and 44.9-48.8 on hipBLASLt; at batch 2048 every shape takes
    the 256 tile, `profiles/r05_35/conv_mm_b*.jsonl`)."""
    if not (_P().own_gemm_conv1x1 and a.is_cuda and a.dtype == torch.bfloat16):
        return 0
    try:
        t = int(lib().gemm_nt_pick(M, N, K))
    except Exception:
        return 0
    if t == 256:
        return 256 if (M // 256) * (N // 256) >= 128 else 0
    return 128 if t == 128 and _P().own_gemm128 else 0


CONV_MM_STATS = {"own": 0, "own128": 0, "blas": 0}   # which path conv_mm took (tests)


def dgrad_wnk(a: torch.Tensor, w2: torch.Tensor, wt: Optional[torch.Tensor]) -> torch.Tensor:
    """conv_mm's weight operand for a 1x1 data gradient a [M, Co] @ W [Co, Ci]: the prefetched
    transpose ``wt`` when gemm.hip takes the GEMM (no transpose launch), else the view ``w2.t()``
    (hipBLASLt then reads W as stored: 892 vs 917 us through a transposed view at the layer-1
    shape, tools/diag/addmm_layout.py)."""
    if wt is not None and _nt_tile(a, a.shape[0], w2.shape[1], w2.shape[0]):
        return wt
    return w2.t()


def conv_mm(a: torch.Tensor, w_nk: torch.Tensor, acc: Optional[torch.Tensor] = None) -> torch.Tensor:
    """a [M, K] @ w_nk^T (+ acc, in place) for a 1x1 conv as a plain GEMM: the forward (w_nk = W
    [Co, C]) or the data gradient (w_nk = W^T [C, Co]; acc = a parked residual gradient). On
    ``gemm.hip`` / ``gemm128.hip`` (NT, acc added in the epilogue: bf16(bf16(a w^T) + acc)) when
    eligible (``_nt_tile``), else hipBLASLt (mm / addmm_ beta = 1). Replaces the layer-3/4
    hipBLASLt GEMMs of the ResNet step (4.8 ms/step in profiles/r04_07/)."""
    M, K = a.shape
    N = w_nk.shape[0]
    tile = _nt_tile(a, M, N, K)
    if (tile and a.is_contiguous() and a.data_ptr() % 16 == 0
            and (acc is None or (acc.is_contiguous() and acc.data_ptr() % 16 == 0))):
        w = (lib().transpose_bf16(w_nk.t()) if (w_nk.stride(0) == 1 and w_nk.dim() == 2)
             else w_nk.contiguous())
        CONV_MM_STATS["own"] += 1
        if tile == 128:
            CONV_MM_STATS["own128"] += 1
        if acc is not None:
            return lib().gemm_nt(a, w, 0, out=acc, cin=acc, tile=tile)
        return lib().gemm_nt(a, w, 0, tile=tile)
    CONV_MM_STATS["blas"] += 1
    if acc is not None:
        return acc.addmm_(a, w_nk.t()) if acc.is_contiguous() else torch.addmm(acc, a, w_nk.t())
    return torch.mm(a, w_nk.t())


def _dgrad(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, stride: int, gemm: bool,
           link, wt: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dX of a 1x1 conv (x only supplies the shape for MIOpen). GEMM path: dX = dY W, with a
    residual gradient parked on ``link`` absorbed by the beta = 1 epilogue."""
    N, C, H, W = x.shape
    Co = w.shape[0]
    if gemm and stride == 1:
        dy2 = dy.permute(0, 2, 3, 1).reshape(N * H * W, Co)
        w2 = w.reshape(Co, C)
        g = link.take() if link is not None else None
        if isinstance(g, MaskedGrad):
            return masked_link_dgrad(dy, w, g, link, wt)
        if isinstance(g, S2Grad):
            if (_P().s2_link_dgrad and dy.dtype == torch.bfloat16 and C % 64 == 0 and Co % 64 == 0
                    and g.H == H and g.W == W):
                if wt is None:
                    wt = w.reshape(Co, C).t().contiguous()
                return lib().conv1x1_link_s2(dy.contiguous(memory_format=torch.channels_last), wt,
                                             g.g)
            g = g.materialize()
        w_nk = dgrad_wnk(dy2, w2, wt)
        if (g is not None and g.dim() == 4 and _P().link_dgrad_plain and dy.dtype == torch.bfloat16
                and g.dtype == torch.bfloat16 and C % 64 == 0 and Co % 64 == 0
                and g.is_contiguous(memory_format=torch.channels_last)
                and not _nt_tile(dy2, N * H * W, C, Co)):
            # the GEMM would go to hipBLASLt (e.g. layer 1.0's 64 -> 64 with the downsample's dX):
            # the fused 1x1 kernel with the parked gradient added in its epilogue instead
            wt2 = wt if wt is not None else w2.t().contiguous()
            return lib().conv1x1_link(dy.contiguous(memory_format=torch.channels_last), wt2, g,
                                      None)[0]
        if g is not None:
            dres = g.permute(0, 2, 3, 1).reshape(N * H * W, C) if g.dim() == 4 else g
            if dres.data_ptr() == g.data_ptr() and dres.is_contiguous():
                d2 = conv_mm(dy2, w_nk, acc=dres)
            else:
                d2 = torch.addmm(dres, dy2, w2)
        else:
            d2 = conv_mm(dy2, w_nk)
        return d2.view(N, H, W, C).permute(0, 3, 1, 2)
    dx, _, _ = torch.ops.aten.convolution_backward(
        dy, x, w, None, [stride, stride], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False])
    return dx


def masked_link_dgrad(dy: torch.Tensor, w: torch.Tensor, mg: MaskedGrad, link,
                      wt: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dX = dY W + m * g of a stride-1 1x1 conv in one kernel (``conv1x1_link``: the masked
    residual gradient is added in the epilogue, never materialised). If the link carries the
    producer's BN context (its bn3 applies its backward in its own convs), the same epilogue
    emits that BN's backward sums over dX and leaves them on the link. ``wt``: W^T [Ci, Co]
    if the forward already has it (``cached_wt``)."""
    Co, Ci = w.shape[0], w.shape[1]
    if wt is None:
        wt = w.reshape(Co, Ci).t().contiguous()
    bctx = link.bn_ctx if link is not None else None
    if bctx is not None:
        z, mask, mean, invstd = bctx
        dx, sdz, sdzx = lib().conv1x1_link(dy, wt, mg.g, mg.mask, z, mask, mean, invstd)
        link.sums = (sdz, sdzx, dx.data_ptr())
        return dx
    return lib().conv1x1_link(dy, wt, mg.g, mg.mask)[0]


def _wgrad(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, stride: int, own: bool,
           pro: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> torch.Tensor:
    """dW of a 1x1 conv. ``pro`` = (sc, bi): the conv's real input is max(x * sc + bi, 0)."""
    if own and stride == 1:
        sc, bi = pro if pro is not None else (None, None)
        return lib().wgrad1x1(dy, x, w.dtype, sc, bi).view_as(w)
    if pro is not None:   # library weight gradient needs the materialised input
        sc, bi = pro
        x = torch.relu(x.float() * sc.view(1, -1, 1, 1) + bi.view(1, -1, 1, 1)).to(x.dtype)
        x = x.contiguous(memory_format=torch.channels_last)
    N, Ci, H, W = x.shape
    if (own and stride == 2 and _P().own_wgrad1x1_s2 and x.is_cuda
            and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16
            and x.is_contiguous(memory_format=torch.channels_last)
            and lib().wgrad3x3s2_ok(N, H, W, dy.shape[1], Ci, 1)):
        # the downsample's weight gradient: the stride-2 DMA kernel with its single tap (2 oh, 2 ow)
        return lib().wgrad3x3s2(dy, x, w.dtype, _zero_row(dy.device), taps=1).reshape(w.shape)
    _, dw, _ = torch.ops.aten.convolution_backward(
        dy, x, w, None, [stride, stride], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False])
    return dw


class _Conv1x1BNStatsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, rmean, rvar, stride, eps, momentum, dgrad_gemm, own_wgrad, link,
                aff=None):
        out = lib().conv1x1_bn_fwd(x, w, None, None, rmean, rmean, rvar, stride, True, eps,
                                   momentum, *(aff or (None, None)))
        y, mean, invstd = out[:3]
        if aff is not None:   # the next BN's affine from the statistics' finalize launch
            _stash_affine(mean, out[3], out[4], aff)
        ctx.wt = cached_wt(w)
        ctx.save_for_backward(x, w)
        ctx.stride, ctx.dgrad_gemm, ctx.own_wgrad, ctx.link = stride, dgrad_gemm, own_wgrad, link
        ctx.mark_non_differentiable(mean, invstd)
        ctx.set_materialize_grads(False)   # no zero-filled grads for the statistics outputs
        return y, mean, invstd

    @staticmethod
    def backward(ctx, dy, _dm, _di):
        x, w = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        # the weight gradient on the side stream (large batches) while the data gradient runs
        dw, h = _wgrad_fork(lambda d, a, b: _wgrad(d, a, b, ctx.stride, ctx.own_wgrad), dy, x, w,
                            conv1x1=True) if ctx.needs_input_grad[1] else (None, None)
        dx = _dgrad(dy, x, w, ctx.stride, ctx.dgrad_gemm, ctx.link, ctx.wt) \
            if ctx.needs_input_grad[0] else None
        dw = _wgrad_join(dw, h)
        return dx, dw, None, None, None, None, None, None, None, None, None


class _BNReLUConv1x1BNStatsFn(torch.autograd.Function):
    """z3 = conv1x1(relu(bn_a(z)), w) with bn_a's batch statistics given (mean, invstd), plus the
    statistics of z3 for the next BN. Gradients for z, bn_a's gamma / beta and w."""

    @staticmethod
    def forward(ctx, z, gamma, beta, mean, invstd, w, rmean, rvar, eps, momentum, dgrad_gemm,
                own_wgrad):
        sc, bi = _affine(gamma, beta, mean, invstd)
        y, m3, i3 = lib().conv1x1_bn_fwd(z, w, sc, bi, rmean, rmean, rvar, 1, True, eps, momentum)
        ctx.save_for_backward(z, gamma, beta, mean, invstd, w, sc, bi)
        ctx.dgrad_gemm, ctx.own_wgrad = dgrad_gemm, own_wgrad
        ctx.mark_non_differentiable(m3, i3)
        ctx.set_materialize_grads(False)   # no zero-filled grads for the statistics outputs
        return y, m3, i3

    @staticmethod
    def backward(ctx, dz3, _dm, _di):
        z, gamma, beta, mean, invstd, w, sc, bi = ctx.saved_tensors
        dz3 = dz3.contiguous(memory_format=torch.channels_last)
        dw = _wgrad(dz3, z, w, 1, ctx.own_wgrad, (sc, bi)) if ctx.needs_input_grad[5] else None
        dy2 = _dgrad(dz3, z, w, 1, ctx.dgrad_gemm, None)
        dz, dg, db, _ = lib().bn_bwd(dy2, None, z, None, gamma, beta, mean, invstd, True, False)
        return dz, dg, db, None, None, dw, None, None, None, None, None, None


class _BNReLUConv1x1BNResFn(torch.autograd.Function):
    """Identity-block tail y = relu(bn3(conv3(relu(bn2(z2)))) + res) with bn3's backward applied
    inside conv3's gradient kernels.

    Forward: the fused conv (bn2 + ReLU prologue, bn3 statistics epilogue) and bn3's apply with
    the residual, keeping bn3's ReLU as a bit mask. Backward: bn3's two sums (from the consumer
    block's conv1 data-gradient epilogue when it left them on ``out_link``, else one reduction
    pass) give per-channel coefficients of dz3 = a (m ? g : 0) + b z3 + c; conv3's data gradient
    (``conv1x1_bnbwd``) and weight gradient (``wgrad1x1`` dz_*) form dz3 while staging, so neither
    dz3 nor the residual gradient is written: the residual gradient m * g is parked on ``res_link``
    as a ``MaskedGrad`` for this block's conv1 data-gradient epilogue."""

    @staticmethod
    def forward(ctx, z, g2, b2, mean2, invstd2, w, g3, b3, res, rmean3, rvar3, eps, momentum,
                res_link, out_link):
        sc, bi = _affine(g2, b2, mean2, invstd2)
        z3, m3, i3 = lib().conv1x1_bn_fwd(z, w, sc, bi, rmean3, rmean3, rvar3, 1, True, eps,
                                          momentum)
        y, _, _, mask = lib().bn_fwd(z3, res, g3, b3, None, None, m3, i3, eps, momentum, True,
                                     False, True)
        ctx.save_for_backward(z, g2, b2, mean2, invstd2, w, sc, bi, z3, mask, g3, b3, m3, i3)
        ctx.res_link, ctx.out_link = res_link, out_link
        if out_link is not None:
            out_link.bn_ctx = (z3, mask, m3, i3)
        return y

    @staticmethod
    def backward(ctx, gy):
        z, g2, b2, mean2, invstd2, w, sc, bi, z3, mask, g3, b3, m3, i3 = ctx.saved_tensors
        gy = gy.contiguous(memory_format=torch.channels_last)
        sums, ol = None, ctx.out_link
        if ol is not None:
            extra = ol.take_tensor()
            if ol.sums is not None and extra is None and ol.sums[2] == gy.data_ptr():
                sums = ol.sums
            ol.sums = ol.bn_ctx = None
            if extra is not None:
                gy = (gy + extra).contiguous(memory_format=torch.channels_last)
        M = gy.numel() // gy.shape[1]
        if sums is None:
            sums = lib().bn_bwd_sums(gy, None, z3, mask, g3, b3, m3, i3, True)
        ca, cb, cc, dg3, db3 = lib().bn_bwd_coeffs(sums[0], sums[1], g3, m3, i3, M)
        Co, Ci = w.shape[0], w.shape[1]
        dw = None
        if ctx.needs_input_grad[5]:
            dw = lib().wgrad1x1(gy, z, w.dtype, sc, bi, z3, mask, ca, cb, cc).view_as(w)
        dy2 = lib().conv1x1_bnbwd(gy, z3, mask, ca, cb, cc, w.reshape(Co, Ci).t().contiguous())
        dz, dg2, db2, _ = lib().bn_bwd(dy2, None, z, None, g2, b2, mean2, invstd2, True, False)
        dres = None
        if ctx.needs_input_grad[8]:
            mg = MaskedGrad(gy, mask)
            if ctx.res_link is not None and not ctx.res_link.closed and ctx.res_link.grad is None:
                ctx.res_link.grad = mg
            else:
                dres = mg.materialize()
        return (dz, dg2, db2, None, None, dw, dg3, db3, dres) + (None,) * 6


def _fin_aff(bn):
    """(gamma, beta) of ``bn`` for a statistics finalize that also writes its affine
    (PerfPolicy.fin_affine, bf16 parameters), else None."""
    g, b = bn.weight, bn.bias
    if (_P().fin_affine and _P().bn_affine_kernel and g is not None and b is not None
            and g.dtype == torch.bfloat16 and b.dtype == torch.bfloat16
            and g.is_contiguous() and b.is_contiguous()):
        return g, b
    return None


def _stash_affine(mean: torch.Tensor, sc: torch.Tensor, bi: torch.Tensor, aff) -> None:
    """Park the finalize's affine (sc, bi) of (gamma, beta) = aff on its mean tensor, for the
    consumer's ``_affine`` (valid while gamma / beta are unchanged: pointer and version checked)."""
    g, b = aff
    mean._cml_affine = (sc, bi, g.data_ptr(), b.data_ptr(), g._version, b._version)


def _cached_affine(gamma: torch.Tensor, beta: torch.Tensor, mean: torch.Tensor):
    a = getattr(mean, "_cml_affine", None)
    if (a is not None and a[2] == gamma.data_ptr() and a[3] == beta.data_ptr()
            and a[4] == gamma._version and a[5] == beta._version):
        return a[0], a[1]
    return None


def _affine(gamma: torch.Tensor, beta: torch.Tensor, mean: torch.Tensor, invstd: torch.Tensor):
    """(sc, bi) = (gamma invstd, beta - mean sc) in fp32: one ``bn_affine`` launch (bit-identical to
    ``gamma.float() * invstd`` and ``beta.float() - mean * sc``, which take five), or none when the
    statistics' finalize already wrote it (``_stash_affine``)."""
    a = _cached_affine(gamma, beta, mean)
    if a is not None:
        return a
    if not _P().bn_affine_kernel:
        sc = gamma.float() * invstd
        return sc, beta.float() - mean * sc
    ab = lib().bn_affine(gamma, beta, mean, invstd)
    return ab[0], ab[1]


def _stats_gram_affine(L, gram, cy, w, M, rmean, rvar, eps, momentum, gamma, beta):
    """``bn_stats_gram`` -> (mean, invstd, sc, bi): the affine from the finalize launch itself
    (bit-identical to ``_affine``) when PerfPolicy.bn_affine_kernel is on, else ``_affine``."""
    if _P().bn_affine_kernel:
        m, i, sc, bi = L.bn_stats_gram(gram, cy, w, M, rmean, rvar, eps, momentum, gamma, beta)
        return m, i, sc, bi
    m, i = L.bn_stats_gram(gram, cy, w, M, rmean, rvar, eps, momentum)
    return (m, i) + _affine(gamma, beta, m, i)


_CONST = {}


def _const(n: int, v: float, device) -> torch.Tensor:
    key = (n, v, device)
    t = _CONST.get(key)
    if t is None:
        t = _CONST[key] = torch.full((n,), v, dtype=torch.float32, device=device)
    return t


# PerfPolicy.gram_stats -- recompute tails: the tail BN's statistics from the Gram matrix of the
# conv input (computed once, reused by the backward) instead of a statistics-only pass of the conv.
# PerfPolicy.cat_bnsums -- recompute tails: bn2's backward sums from the epilogue of the GEMM that
# produces its output gradient dy2 (``conv1x1_cat_bnsums``, ReLU mask recomputed from z2), so only
# bn2's apply pass remains; up to cat_bnsums_maxc channels (round 2: the register-staged sums
# variant ran MT = 1 tiles, which on the 128 / 256-channel GEMMs cost about what the reduction pass
# did: profiles/r02_prof53_*).


def scaled_cat(w1: torch.Tensor, s1: torch.Tensor, w2: torch.Tensor, s2: torch.Tensor):
    """bf16 [Co, K1 + K2] = [diag(s1) w1 | diag(s2) w2] (w bf16 [Co, K], s fp32 [Co]): each product
    in fp32, rounded once into its half of the output -- two launches, bit-identical to
    ``torch.cat([w1.float() * s1[:, None], w2.float() * s2[:, None]], 1).to(torch.bfloat16)``
    (six)."""
    k1 = w1.shape[1]
    out = torch.empty(w1.shape[0], k1 + w2.shape[1], dtype=torch.bfloat16, device=w1.device)
    torch.mul(w1, s1[:, None], out=out[:, :k1])
    torch.mul(w2, s2[:, None], out=out[:, k1:])
    return out


def fold_cat(w1: torch.Tensor, a: torch.Tensor, c: torch.Tensor, w2: torch.Tensor):
    """Weights and bias of a two-source GEMM whose first source is a BN + ReLU backward,
    a (mask ? g : 0) + c (a, c fp32 [K1]; w1 [Co, K1], w2 [Co, K2] fp32): the kernels stage only
    (mask ? g : 0), so a is folded into w1's columns and c into a per-output bias,
    [a u + c | x2] [w1 | w2]^T = [u | x2] [w1 diag(a) | w2]^T + w1 c.
    Returns (w_cat bf16 [Co, K1 + K2] contiguous, bias fp32 [Co])."""
    w_cat = torch.cat([w1 * a[None, :], w2], 1).to(torch.bfloat16).contiguous()
    return w_cat, torch.mv(w1, c)


def _own_dgb(gamma: torch.Tensor, beta: torch.Tensor) -> bool:
    """Whether a BN's parameter gradients come out of its backward sums' finalize launch (bf16
    parameters: the values ``bn_bwd_coeffs`` rounds, without its launch;
    PerfPolicy.fin_dgamma)."""
    return (_P().fin_dgamma and gamma.dtype == torch.bfloat16 and beta.dtype == torch.bfloat16
            and gamma.is_contiguous() and beta.is_contiguous())


def _cat_dgrad_bn2(L, gy, mask, z, sc, bi, w_cat, bias, g2, b2, mean2, invstd2):
    """dy2 = [(mask ? gy : 0) | relu(z sc + bi)] w_cat^T + bias (``fold_cat``), then bn2's
    (BN + ReLU on z) backward: (dz, dgamma2, dbeta2)."""
    pol = _P()
    if pol.cat_bnsums and z.shape[1] <= pol.cat_bnsums_maxc:
        if _own_dgb(g2, b2):   # bn2's parameter gradients from the sums' finalize launch
            dg2, db2 = torch.empty_like(g2), torch.empty_like(b2)
            dy2, s2, q2 = L.conv1x1_cat_bnsums(gy, mask, z, sc, bi, w_cat, bias, mean2, invstd2,
                                               dg2, db2)
        else:
            dy2, s2, q2 = L.conv1x1_cat_bnsums(gy, mask, z, sc, bi, w_cat, bias, mean2, invstd2)
            M = z.numel() // z.shape[1]
            _, _, _, dg2, db2 = L.bn_bwd_coeffs(s2, q2, g2, mean2, invstd2, M)
        return L.bn_bwd_apply(dy2, z, g2, b2, mean2, invstd2, s2, q2), dg2, db2
    dy2 = L.conv1x1_cat(gy, mask, z, sc, bi, w_cat, bias)
    dz, dg2, db2, _ = L.bn_bwd(dy2, None, z, None, g2, b2, mean2, invstd2, True, False)
    return dz, dg2, db2


class _RecomputeTailFn(torch.autograd.Function):
    """Identity-block tail y = relu(bn3(conv3(relu(bn2(z2)))) + res) that never stores z3.

    z3 = conv3(y2) (y2 = relu(bn2(z2)), p channels) has 4p channels, so in the layer-1/2 blocks
    writing it and reading it back (forward apply, bn3's backward sums, conv3's two gradient
    GEMMs) is most of the tail's HBM traffic. Here:

    Forward: bn3's statistics from y2's Gram matrix: mean = W3 sum(y2) / M, var = w^T (y2^T y2)
    w / M - mean^2 per output channel (``wgrad1x1_ex`` mode 3 + ``bn_stats_gram``; p x p instead
    of the 4p-channel conv, and the Gram is the one the backward needs anyway), then the GEMM with
    bn3 + residual + ReLU applied in its epilogue (``conv1x1_bnres``, y and its bit mask).
    PerfPolicy.gram_stats off: a statistics-only pass of the conv instead (bn3 statistics of the bf16
    products).

    Backward, with u = m * g (g the block-output gradient, m bn3's ReLU mask) and
    dz3 = a u + b z3 + c (bn3's backward: a = gamma invstd, b, c from its sums):
      P = u^T y2 and s = sum u           one weight-gradient pass (``wgrad1x1_ex`` mode 2 + column
                                         sums), reading g, m and z2 -- not z3
      Gram = y2^T y2, sum y2             one small pass over z2 (mode 3)
      q = sum u (z3 - mean) invstd = invstd (rowsum(W3 * P) - mean s)    (z3 = y2 W3^T)
      dW3 = diag(a) P + diag(b) W3 Gram + c (sum y2)^T
      dy2 = (a u + c) W3 + y2 (W3^T diag(b) W3)     one two-source GEMM (``conv1x1_cat``, K = 5p)
    All exact identities of the unfused computation (z3 in fp32 instead of its bf16 rounding).
    The residual gradient m * g is parked on ``res_link`` as a ``MaskedGrad`` as in
    ``_BNReLUConv1x1BNResFn``."""

    @staticmethod
    def forward(ctx, z, g2, b2, mean2, invstd2, w, g3, b3, res, rmean3, rvar3, eps, momentum,
                res_link, out_link):
        sc, bi = _affine(g2, b2, mean2, invstd2)
        wc = w.contiguous()
        L = lib()
        gram = cy = None
        if _P().gram_stats:
            # bn3's statistics from y2's Gram matrix (also the backward's), not a conv pass; bn3's
            # affine from the same finalize launch
            gram, cy = L.wgrad1x1_ex(z, z, sc, bi, 3, None, sc, bi, None, True)
            m3, i3, sc3, bi3 = _stats_gram_affine(L, gram, cy, wc, z.numel() // z.shape[1], rmean3,
                                                  rvar3, eps, momentum, g3, b3)
        else:
            m3, i3 = L.conv1x1_bn_stats_only(z, wc, sc, bi, rmean3, rmean3, rvar3, eps, momentum)
            sc3, bi3 = _affine(g3, b3, m3, i3)
        y, mask = L.conv1x1_bnres(z, wc, sc, bi, sc3, bi3, res)
        ctx.gram = (gram, cy)
        ctx.save_for_backward(z, g2, b2, mean2, invstd2, w, sc, bi, mask, g3, m3, i3)
        ctx.res_link, ctx.out_link = res_link, out_link
        if out_link is not None:
            out_link.bn_ctx = None   # the consumer's conv1 epilogue owes this tail no sums
        return y

    @staticmethod
    def backward(ctx, gy):
        z, g2, b2, mean2, invstd2, w, sc, bi, mask, g3, m3, i3 = ctx.saved_tensors
        gy = gy.contiguous(memory_format=torch.channels_last)
        ol = ctx.out_link
        if ol is not None:
            extra = ol.take_tensor()
            ol.sums = ol.bn_ctx = None
            if extra is not None:
                gy = (gy + extra).contiguous(memory_format=torch.channels_last)
        M = gy.numel() // gy.shape[1]
        Co = w.shape[0]
        dev = gy.device
        L = lib()
        P, s = L.wgrad1x1_ex(gy, z, sc, bi, 2, mask, _const(Co, 1.0, dev), None,
                             _const(Co, 0.0, dev), True)
        gram, cy = ctx.gram
        ctx.gram = None
        if gram is None:
            gram, cy = L.wgrad1x1_ex(z, z, sc, bi, 3, None, sc, bi, None, True)
        # q, bn3's coefficients, dW3 = diag(a) P + diag(b) W3 Gram + c cy^T and the folded
        # w_cat = [W3^T diag(a) | W3^T diag(b) W3], bias = W3^T c: two launches (tail_prep.hip)
        need_dw = ctx.needs_input_grad[5]
        w_cat, bias, dw, dg3, db3 = L.tail_bwd_prep(w.contiguous(), P, s, gram, cy, g3, m3, i3, M,
                                                    need_dw)
        dw = dw.view_as(w) if need_dw else None
        dz, dg2, db2 = _cat_dgrad_bn2(L, gy, mask, z, sc, bi, w_cat, bias, g2, b2, mean2, invstd2)
        dres = None
        if ctx.needs_input_grad[8]:
            mg = MaskedGrad(gy, mask)
            if ctx.res_link is not None and not ctx.res_link.closed and ctx.res_link.grad is None:
                ctx.res_link.grad = mg
            else:
                dres = mg.materialize()
        return (dz, dg2, db2, None, None, dw, dg3, db3, dres) + (None,) * 6


class _RecomputeDownTailFn(torch.autograd.Function):
    """Downsample-block tail y = relu(bn3(conv3(relu(bn2(z2)))) + bnd(convd(x))) with stride-1
    convd, storing neither z3 nor zd (both 4p channels; ResNet-50 layer 1: 3.3 GB each at batch
    2048).

    Forward: statistics-only passes of both convs, then one GEMM over [y2 | x] (K = p + Cin)
    with the BN scales folded into the weights, + both BN shifts, ReLU and its mask
    (``conv1x1_cat_bnres``). Backward as ``_RecomputeTailFn`` for each branch -- both BNs see the
    same u = m * g -- with dx = (ad u + cd) Wd + x (Wd^T diag(bd) Wd) from ``conv1x1_cat`` (its
    second source stages x as is, as the forward's GEMM does: x is a ReLU output, as every block
    input is). x's gradient goes back through autograd (callers wrap x in ``link_tap`` to hand it
    to conv1's data-gradient GEMM)."""

    @staticmethod
    def forward(ctx, z, g2, b2, mean2, invstd2, w3, g3, b3, rm3, rv3, x, wd, gd, bd, rmd, rvd,
                eps, momentum, out_link):
        sc, bi = _affine(g2, b2, mean2, invstd2)
        L = lib()
        w3c, wdc = w3.contiguous(), wd.contiguous()
        grams = (None, None, None, None)
        if _P().gram_stats:
            M_ = z.numel() // z.shape[1]
            gram3, cy = L.wgrad1x1_ex(z, z, sc, bi, 3, None, sc, bi, None, True)
            gramd, cx = L.wgrad1x1_ex(x, x, None, None, 0, None, None, None, None, True)
            m3, i3, sc3, bi3 = _stats_gram_affine(L, gram3, cy, w3c, M_, rm3, rv3, eps, momentum,
                                                  g3, b3)
            md, idd, scd, bid = _stats_gram_affine(L, gramd, cx, wdc, M_, rmd, rvd, eps, momentum,
                                                   gd, bd)
            grams = (gram3, cy, gramd, cx)
        else:
            m3, i3 = L.conv1x1_bn_stats_only(z, w3c, sc, bi, rm3, rm3, rv3, eps, momentum)
            md, idd = L.conv1x1_bn_stats_only(x, wdc, None, None, rmd, rmd, rvd, eps, momentum)
            sc3, bi3 = _affine(g3, b3, m3, i3)
            scd, bid = _affine(gd, bd, md, idd)
        ctx.grams = grams
        Co, P_, Cin = w3.shape[0], w3.shape[1], wd.shape[1]
        if z.is_cuda and w3c.dtype == torch.bfloat16 and wdc.dtype == torch.bfloat16:
            # both halves and the bias sum in one launch (bit-identical to the three below)
            w_cat, bias = L.scaled_cat_bias(w3c.view(Co, P_), sc3, wdc.view(Co, Cin), scd, bi3,
                                            bid)
        else:
            bias = bi3 + bid
            w_cat = scaled_cat(w3c.view(Co, P_), sc3, wdc.view(Co, Cin), scd)
        dev = z.device
        # x: the block input, a ReLU output, staged as is
        y, mask = L.conv1x1_cat_bnres(z, x, sc, bi, None, None, w_cat,
                                      _const(Co, 1.0, dev), bias)
        ctx.save_for_backward(z, g2, b2, mean2, invstd2, w3, sc, bi, mask, g3, m3, i3, x, wd, gd,
                              md, idd)
        ctx.out_link = out_link
        if out_link is not None:
            out_link.bn_ctx = None
        return y

    @staticmethod
    def backward(ctx, gy):
        (z, g2, b2, mean2, invstd2, w3, sc, bi, mask, g3, m3, i3, x, wd, gd, md,
         idd) = ctx.saved_tensors
        gy = gy.contiguous(memory_format=torch.channels_last)
        ol = ctx.out_link
        if ol is not None:
            extra = ol.take_tensor()
            ol.sums = ol.bn_ctx = None
            if extra is not None:
                gy = (gy + extra).contiguous(memory_format=torch.channels_last)
        M = gy.numel() // gy.shape[1]
        Co = w3.shape[0]
        dev = gy.device
        L = lib()
        one, zero = _const(Co, 1.0, dev), _const(Co, 0.0, dev)
        P3, s = L.wgrad1x1_ex(gy, z, sc, bi, 2, mask, one, None, zero, True)
        Pd, _ = L.wgrad1x1_ex(gy, x, None, None, 2, mask, one, None, zero, False)
        gram3, cy, gramd, cx = ctx.grams
        ctx.grams = None
        if gram3 is None:
            gram3, cy = L.wgrad1x1_ex(z, z, sc, bi, 3, None, sc, bi, None, True)
            gramd, cx = L.wgrad1x1_ex(x, x, None, None, 0, None, None, None, None, True)
        # each branch's backward algebra in two launches (tail_prep.hip; see _RecomputeTailFn)
        nd3, ndd = ctx.needs_input_grad[5], ctx.needs_input_grad[11]
        w_cat3, bias3, dw3, dg3, db3 = L.tail_bwd_prep(w3.contiguous(), P3, s, gram3, cy, g3, m3,
                                                       i3, M, nd3)
        w_catd, biasd, dwd, dgd, dbd = L.tail_bwd_prep(wd.contiguous(), Pd, s, gramd, cx, gd, md,
                                                       idd, M, ndd)
        dw3 = dw3.view_as(w3) if nd3 else None
        dwd = dwd.view_as(wd) if ndd else None
        dz, dg2, db2 = _cat_dgrad_bn2(L, gy, mask, z, sc, bi, w_cat3, bias3, g2, b2, mean2,
                                      invstd2)
        dx = None
        if ctx.needs_input_grad[10]:
            dx = L.conv1x1_cat(gy, mask, x, None, None, w_catd, biasd)   # x staged as is
        return (dz, dg2, db2, None, None, dw3, dg3, db3, None, None, dx, dwd, dgd, dbd) + \
            (None,) * 5


class _Subsample2Fn(torch.autograd.Function):
    """x[:, :, ::2, ::2] as a dense NHWC tensor (the pixels a stride-2 1x1 conv reads); backward
    scatters the gradient back into a zero-filled full-resolution tensor."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        if x.is_cuda and x.dtype == torch.bfloat16 and x.shape[1] % 8 == 0:
            return lib().subsample2(x.contiguous(memory_format=torch.channels_last))
        return x[:, :, ::2, ::2].contiguous(memory_format=torch.channels_last)

    @staticmethod
    def backward(ctx, g):
        N, C, H, W = ctx.shape
        if g.is_cuda and g.dtype == torch.bfloat16 and C % 8 == 0:
            return lib().upsample2_scatter(g, H, W)
        dx = torch.zeros(ctx.shape, dtype=g.dtype, device=g.device).contiguous(
            memory_format=torch.channels_last)
        dx[:, :, ::2, ::2] = g
        return dx


def subsample2(x: torch.Tensor) -> torch.Tensor:
    return _Subsample2Fn.apply(x)


class S2Grad:
    """A stride-2 conv's data gradient left compact ([N, C, ceil(H/2), ceil(W/2)]): the parallel
    1x1 data-gradient kernel adds it at the even pixels (``conv1x1_link_s2``); anything else
    calls ``materialize`` (zero-filled full resolution)."""
    __slots__ = ("g", "H", "W")

    def __init__(self, g: torch.Tensor, H: int, W: int):
        self.g, self.H, self.W = g, H, W

    def materialize(self) -> torch.Tensor:
        return lib().upsample2_scatter(self.g, self.H, self.W)


class _Subsample2LinkFn(torch.autograd.Function):
    """``subsample2`` whose backward parks the compact gradient on a ResidualLink (for conv1's
    data-gradient kernel to add at the even pixels) instead of scattering it; if the consumer
    already ran, the scattered gradient flows normally."""

    @staticmethod
    def forward(ctx, x, link):
        ctx.shape, ctx.link = x.shape, link
        return lib().subsample2(x.contiguous(memory_format=torch.channels_last))

    @staticmethod
    def backward(ctx, g):
        link = ctx.link
        g = g.contiguous(memory_format=torch.channels_last)
        if link.closed or link.grad is not None:
            return lib().upsample2_scatter(g, ctx.shape[2], ctx.shape[3]), None
        link.grad = S2Grad(g, ctx.shape[2], ctx.shape[3])
        return None, None


def subsample2_link(x: torch.Tensor, link) -> torch.Tensor:
    """``subsample2(x)`` with the backward hand-off of _Subsample2LinkFn (GPU bf16 NHWC)."""
    if link is None or not (x.is_cuda and x.dtype == torch.bfloat16 and x.shape[1] % 8 == 0):
        return subsample2(x)
    return _Subsample2LinkFn.apply(x, link)


def down_tail_recompute_s2_ok(x: torch.Tensor, planes: int, down_conv) -> bool:
    """Stride-2 downsample tails (ResNet-50 layer 2) on the recompute kernels: the convolution
    reads x[:, :, ::2, ::2], materialised once (``subsample2``), so the stride-1 kernels apply."""
    pol = _P()
    return (pol.recompute_down_tail_s2 and down_conv.stride[0] == 2 and down_conv.stride[1] == 2
            and planes in (64, 128, 256, 512) and x.shape[1] % 64 == 0
            and x.shape[1] <= pol.down_tail_s2_max_cin)


# PerfPolicy.s2_link_dgrad -- stride-2 downsample tails: the compact data gradient is added at the
# even pixels by conv1's data-gradient kernel (off: scattered to full resolution, then addmm_).
# PerfPolicy.recompute_down_tail_s2 / down_tail_s2_max_cin -- widest block input of a recompute
# stride-2 downsample tail (256: layer 2; 512: also layer 3, step 128.9 / 129.2 -> 128.0 / 128.5 ms
# and -1.1 GiB peak, profiles/r02_down_tail_l3_58/).


def down_tail_recompute_ok(x: torch.Tensor, planes: int, down_conv) -> bool:
    """Stride-1 downsample convs (ResNet-50 layer 1) with the recompute kernels' channel counts."""
    return (down_conv.stride[0] == 1 and planes in (64, 128) and x.shape[1] % 64 == 0
            and x.shape[1] <= 256)


def down_tail_recompute(z: torch.Tensor, bn_a, stats_a, conv, bn_b, x: torch.Tensor, down_conv,
                        down_bn, out_link=None) -> torch.Tensor:
    """y = relu(bn_b(conv(relu(bn_a(z)))) + down_bn(down_conv(x))) (see _RecomputeDownTailFn)."""
    mean, invstd = stats_a
    return _RecomputeDownTailFn.apply(z, bn_a.weight, bn_a.bias, mean, invstd, conv.weight,
                                      bn_b.weight, bn_b.bias, bn_b.running_mean,
                                      bn_b.running_var, x, down_conv.weight, down_bn.weight,
                                      down_bn.bias, down_bn.running_mean, down_bn.running_var,
                                      bn_b.eps, bn_b.momentum, out_link)


def recompute_tail_ok(planes: int) -> bool:
    """Channel counts of the recompute tail's kernels (every ResNet-50 stage)."""
    return planes in (64, 128, 256, 512)


def bnrelu_conv1x1_bn_res_recompute(z: torch.Tensor, bn_a, stats_a, conv, bn_b,
                                    res: torch.Tensor, res_link=None,
                                    out_link=None) -> torch.Tensor:
    """``bnrelu_conv1x1_bn_res`` without a stored z3 (see _RecomputeTailFn)."""
    mean, invstd = stats_a
    return _RecomputeTailFn.apply(z, bn_a.weight, bn_a.bias, mean, invstd, conv.weight,
                                  bn_b.weight, bn_b.bias, res, bn_b.running_mean,
                                  bn_b.running_var, bn_b.eps, bn_b.momentum, res_link, out_link)


def res_tail_ok(planes: int) -> bool:
    """Channel counts the fused identity tail's kernels take (every ResNet-50 stage)."""
    return planes % 64 == 0 and planes * 4 <= 2048


def bnrelu_conv1x1_bn_res(z: torch.Tensor, bn_a, stats_a, conv, bn_b, res: torch.Tensor,
                          res_link=None, out_link=None) -> torch.Tensor:
    """y = relu(bn_b(conv(relu(bn_a(z)))) + res) for an identity block (training, GPU bf16);
    bn_a's batch statistics ``stats_a`` from ``bn_stats``; bn_b's running statistics are
    updated. See _BNReLUConv1x1BNResFn for the backward."""
    mean, invstd = stats_a
    return _BNReLUConv1x1BNResFn.apply(z, bn_a.weight, bn_a.bias, mean, invstd, conv.weight,
                                       bn_b.weight, bn_b.bias, res, bn_b.running_mean,
                                       bn_b.running_var, bn_b.eps, bn_b.momentum, res_link,
                                       out_link)


_ZERO_ROWS = {}


def _zero_row(device: torch.device) -> torch.Tensor:
    """A cached row of zeros (padding source of conv_gemm's gathered loads)."""
    z = _ZERO_ROWS.get(device)
    if z is None:
        z = _ZERO_ROWS[device] = torch.zeros(256, dtype=torch.bfloat16, device=device)
    return z


# PerfPolicy.side_wgrad: a weight gradient depends only on the conv's output gradient and saved
# input, so it can run on a second HIP stream while the data-gradient and BN-backward kernels of
# the same conv run on the current one (the GPU fills one kernel's tail rounds with the other's
# workgroups). The side stream first waits for the current stream; the current stream waits for
# the side stream before the backward returns, so every tensor the side kernels touch stays
# ordered with the caching allocator's reuse on the current stream.
_SIDE_STREAMS: Dict[torch.device, "torch.cuda.Stream"] = {}


def _wgrad_fork(fn, *args, conv1x1: bool = False):
    """(dw, handle): ``fn(*args)`` on the side stream (PerfPolicy.side_wgrad, CUDA tensors, batch
    ``args[0].shape[0]`` >= side_wgrad_min_batch), else inline (handle None). ``_wgrad_join``
    before the backward returns."""
    dev = args[0].device
    pol = _P()
    if not (pol.side_wgrad and dev.type == "cuda" and args[0].shape[0] >= pol.side_wgrad_min_batch
            and (pol.side_wgrad_1x1 or not conv1x1)):
        return fn(*args), None
    side = _SIDE_STREAMS.get(dev)
    if side is None:
        side = _SIDE_STREAMS[dev] = torch.cuda.Stream(device=dev)
    main = torch.cuda.current_stream(dev)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        dw = fn(*args)
    return dw, (main, side)


def _wgrad_join(dw: Optional[torch.Tensor], handle) -> Optional[torch.Tensor]:
    if handle is None:
        return dw
    main, side = handle
    main.wait_stream(side)
    if dw is not None:
        dw.record_stream(main)   # allocated on the side stream, consumed on the current one
    return dw


# PerfPolicy.own_wgrad3x3 -- 3x3 weight gradients on csrc/kernels/wgrad3x3.hip (nine taps per
# workgroup): 1.4-2.0x faster than MIOpen's at the ResNet-50 shapes (profiles/r02_wgrad3x3_39.jsonl)


def _wgrad3x3(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    N, Ci, H, W = x.shape
    Co = dy.shape[1]
    if _P().own_wgrad3x3 and lib().wgrad3x3_direct_ok(N, H, W, Co, Ci):
        return lib().wgrad3x3(dy, x, w.dtype, _zero_row(dy.device))
    return torch.ops.aten.convolution_backward(
        dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])[1]


_WL_BATCH = {}   # id(weight) -> (weight, wf, wr): this forward's prefetched weight layouts


def prefetch_wlayouts(ws) -> bool:
    """Make the GEMM layouts of all bf16 GPU conv weights ``ws`` in one launch
    (``conv_wlayouts_multi``) for the forward about to run: 3x3 weights' ``_w3x3_layouts``, 1x1
    weights' transposes W^T (``cached_wt``: the 1x1 data-gradient operand, which the conv's
    forward keeps for its backward). The caller clears them with ``clear_wlayouts`` when the
    forward ends (the weights must not change in between). False (nothing done) for fewer than
    two eligible weights."""
    ws = [w for w in ws if w.is_cuda and w.dtype == torch.bfloat16 and w.dim() == 4
          and w.shape[2] == w.shape[3] and w.shape[2] in (1, 3)]
    if len(ws) < 2:
        return False
    for w, (wf, wr) in zip(ws, lib().conv_wlayouts_multi(ws)):
        _WL_BATCH[id(w)] = (w, wf, wr)
    return True


def clear_wlayouts() -> None:
    _WL_BATCH.clear()


def cached_wt(w: torch.Tensor) -> Optional[torch.Tensor]:
    """W^T [Ci, Co] of a prefetched 1x1 weight (``prefetch_wlayouts``), else None."""
    e = _WL_BATCH.get(id(w))
    return e[2] if e is not None and e[0] is w and w.shape[2] == 1 else None


def _w3x3_layouts(w: torch.Tensor, want_wf: bool):
    """(wf or None, wr): the implicit-GEMM forward layout wf [Co, 9 Ci] (k = (3 ky + kx) Ci + ci)
    and the data-gradient layout wr [Ci, 9 Co] (rotated, transposed: wr[ci][(3 ky + kx) Co + co] =
    w[co][ci][2 - ky][2 - kx]) of a 3x3 weight, in one launch (``conv3x3_wlayouts``) instead of a
    permute copy, a flip and another permute copy per conv and step -- or none when the model's
    forward prefetched every block's layouts together (``prefetch_wlayouts``)."""
    e = _WL_BATCH.get(id(w))
    if e is not None and e[0] is w:
        return (e[1] if want_wf else None), e[2]
    if w.is_cuda and w.dtype == torch.bfloat16:
        wf, wr = lib().conv3x3_wlayouts(w, want_wf)
        return wf, wr
    Co, Ci = w.shape[0], w.shape[1]
    wf = w.permute(0, 2, 3, 1).reshape(Co, 9 * Ci).contiguous() if want_wf else None
    return wf, w.flip(2, 3).permute(1, 2, 3, 0).reshape(Ci, 9 * Co).contiguous()


class _Conv3x3Fn(torch.autograd.Function):
    """3x3 / stride 1 / padding 1 conv: forward on MIOpen, data gradient on ``conv_gemm.hip`` (the
    forward implicit GEMM of dy with the rotated, transposed weights; 15-27 % faster than MIOpen's
    backward-data at the ResNet-50 shapes, profiles/r02_conv_gemm24/), weight gradient on
    ``wgrad3x3.hip``."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return F.conv2d(x, w, padding=1)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            # w_rot[ci][ky][kx][co] = w[co][ci][2 - ky][2 - kx], flattened k = tap Co + co
            wr = getattr(ctx, "wr", None)
            if wr is None:
                wr = _w3x3_layouts(w, False)[1]
            dx = lib().conv_gemm(dy, wr, 9, _zero_row(dy.device))
        if ctx.needs_input_grad[1]:
            dw = _wgrad3x3(dy, x, w)
        return dx, dw


class _Conv3x3BNStatsFn(torch.autograd.Function):
    """(z, mean, invstd): 3x3 / stride 1 / padding 1 conv on ``conv_gemm.hip`` with the next BN's
    training statistics accumulated in its epilogue (no separate statistics pass over z); backward
    as ``_Conv3x3Fn``."""

    @staticmethod
    def forward(ctx, x, w, rmean, rvar, eps, momentum, aff=None):
        wf, wr = _w3x3_layouts(w, True)   # both layouts now: the backward reuses wr
        y, mean, invstd = _conv_gemm_bn(x, wf, rmean, rvar, eps, momentum, 1, aff)
        ctx.save_for_backward(x, w)
        ctx.wr = wr
        ctx.mark_non_differentiable(mean, invstd)
        ctx.set_materialize_grads(False)   # no zero-filled grads for the statistics outputs
        return y, mean, invstd

    @staticmethod
    def backward(ctx, dy, _dm, _di):
        dx, dw = _Conv3x3Fn.backward(ctx, dy)
        return dx, dw, None, None, None, None, None


def _conv_gemm_bn(x, wf, rmean, rvar, eps, momentum, stride, aff):
    """``conv_gemm_bn`` (3x3 taps) -> (y, mean, invstd); with aff = (gamma, beta) the next BN's
    affine comes out of the same finalize launch and is parked on mean (``_stash_affine``)."""
    out = lib().conv_gemm_bn(x, wf, 9, _zero_row(x.device), rmean, rmean, rvar, eps, momentum,
                             stride, *(aff or (None, None)))
    if aff is not None:
        _stash_affine(out[1], out[3], out[4], aff)
    return out[0], out[1], out[2]


class _BNReLUConv3x3BNStatsFn(torch.autograd.Function):
    """(z2, mean2, invstd2) = conv3x3(relu(bn1(z1))) and bn2's training statistics, with bn1's
    batch statistics (mean1, invstd1) given by its producer. Forward as ``bn_act`` +
    ``_Conv3x3BNStatsFn`` (y1 is materialised: the implicit GEMM stages it with global_load_lds).
    Backward: the 3x3 data-gradient GEMM also takes bn1's BN + ReLU backward sums in its epilogue
    (``conv_gemm_bnsums``, ReLU bit recomputed from z1), so bn1's backward is its apply pass only
    (the separate reduction re-read dy1 and z1)."""

    @staticmethod
    def forward(ctx, z1, g1, b1, mean1, invstd1, eps1, w, rmean, rvar, eps, momentum, aff=None):
        L = lib()
        y1 = L.bn_fwd(z1, None, g1, b1, None, None, mean1, invstd1, eps1, momentum, True, False,
                      False)[0]
        wf, wr = _w3x3_layouts(w, True)   # both layouts now: the backward reuses wr
        z2, m2, i2 = _conv_gemm_bn(y1, wf, rmean, rvar, eps, momentum, 1, aff)
        ctx.save_for_backward(z1, g1, b1, mean1, invstd1, y1, w)
        ctx.wr = wr
        ctx.aff1 = _cached_affine(g1, b1, mean1)   # bn1's affine, for the backward
        ctx.mark_non_differentiable(m2, i2)
        ctx.set_materialize_grads(False)   # no zero-filled grads for the statistics outputs
        return z2, m2, i2

    @staticmethod
    def backward(ctx, dz2, _dm, _di):
        z1, g1, b1, mean1, invstd1, y1, w = ctx.saved_tensors
        dz2 = dz2.contiguous(memory_format=torch.channels_last)
        L = lib()
        wr = ctx.wr   # rotated / transposed layout, made by the forward
        dw, h = _wgrad_fork(_wgrad3x3, dz2, y1, w) if ctx.needs_input_grad[6] else (None, None)
        sc, bi = ctx.aff1 or _affine(g1, b1, mean1, invstd1)
        # bn1's parameter gradients come out of the sums' finalize launch (no bn_bwd_coeffs)
        own_dgb = g1.dtype == torch.bfloat16 and b1.dtype == torch.bfloat16
        dg1, db1 = (torch.empty_like(g1), torch.empty_like(b1)) if own_dgb else (None, None)
        dy1, s1, q1 = L.conv_gemm_bnsums(dz2, wr, 9, _zero_row(dz2.device), z1, sc, bi, mean1,
                                         invstd1, dg1, db1)
        if not own_dgb:
            M = z1.numel() // z1.shape[1]
            _, _, _, dg1, db1 = L.bn_bwd_coeffs(s1, q1, g1, mean1, invstd1, M)
        dz1 = L.bn_bwd_apply(dy1, z1, g1, b1, mean1, invstd1, s1, q1)
        dw = _wgrad_join(dw, h)
        return dz1, dg1, db1, None, None, None, dw, None, None, None, None, None


def _wgrad3x3_s2(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """Weight gradient of a stride-2 / padding-1 3x3 conv: ``wgrad3x3s2`` (wgrad1x1.hip's LDS-DMA
    kernel on the implicit im2col of x, the padding rows gathered from a zero row) when the shape
    has a plan and PerfPolicy.own_wgrad3x3_s2 is on, else MIOpen. (An own nine-tap kernel over the
    raw input rows measured 1.1-1.45x slower than MIOpen, docs/HISTORY.md "Round 4".)
    Batch 2048 (profiles/r05_16/): 256 -> 256 at 28 x 28 585-603 us vs MIOpen 692-704, 512 -> 512
    at 14 x 14 555-603 vs 644-674; the 128-channel layer-2 conv (128 x 128 tiles, x gathered 2.25x
    and dy re-read per tap through L2) 969 vs 850 stays on MIOpen (Ci < 256)."""
    N, Ci, H, W = x.shape
    if (_P().own_wgrad3x3_s2 and Ci >= _P().wgrad3x3_s2_min_ci and x.is_cuda
            and dy.dtype == torch.bfloat16
            and x.dtype == torch.bfloat16
            and lib().wgrad3x3s2_ok(N, H, W, dy.shape[1], Ci)):
        return lib().wgrad3x3s2(dy, x.contiguous(memory_format=torch.channels_last), w.dtype,
                                _zero_row(dy.device))
    return torch.ops.aten.convolution_backward(
        dy, x, w, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])[1]


class _Conv3x3S2BNStatsFn(torch.autograd.Function):
    """(z, mean, invstd): stride-2 / padding-1 3x3 conv on ``conv_gemm.hip`` (stride-2 gather)
    with the next BN's statistics in the epilogue. Backward: the data gradient as four
    output-parity-class implicit GEMMs of 4 / 2 / 2 / 1 taps (``conv_gemm_s2dgrad``: no multiply
    by the structural zeros of a stride-2 transposed conv, every dx pixel written once, no fill);
    weight gradient on MIOpen."""

    @staticmethod
    def forward(ctx, x, w, rmean, rvar, eps, momentum, aff=None):
        wf, wr = _w3x3_layouts(w, True)
        y, mean, invstd = _conv_gemm_bn(x, wf, rmean, rvar, eps, momentum, 2, aff)
        ctx.save_for_backward(x, w)
        ctx.wr = wr
        ctx.mark_non_differentiable(mean, invstd)
        ctx.set_materialize_grads(False)
        return y, mean, invstd

    @staticmethod
    def backward(ctx, dy, _dm, _di):
        x, w = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = lib().conv_gemm_s2dgrad(dy, ctx.wr, _zero_row(dy.device))[0] \
            if ctx.needs_input_grad[0] else None
        dw = _wgrad3x3_s2(dy, x, w) if ctx.needs_input_grad[1] else None
        return dx, dw, None, None, None, None, None


class _BNReLUConv3x3S2BNStatsFn(torch.autograd.Function):
    """``_BNReLUConv3x3BNStatsFn`` for the stride-2 3x3 conv of a downsample block: the
    parity-class data gradient also takes bn1's BN + ReLU backward sums in its epilogue, so bn1's
    backward is its apply pass only."""

    @staticmethod
    def forward(ctx, z1, g1, b1, mean1, invstd1, eps1, w, rmean, rvar, eps, momentum, aff=None):
        L = lib()
        y1 = L.bn_fwd(z1, None, g1, b1, None, None, mean1, invstd1, eps1, momentum, True, False,
                      False)[0]
        wf, wr = _w3x3_layouts(w, True)
        z2, m2, i2 = _conv_gemm_bn(y1, wf, rmean, rvar, eps, momentum, 2, aff)
        ctx.save_for_backward(z1, g1, b1, mean1, invstd1, y1, w)
        ctx.wr = wr
        ctx.aff1 = _cached_affine(g1, b1, mean1)
        ctx.mark_non_differentiable(m2, i2)
        ctx.set_materialize_grads(False)
        return z2, m2, i2

    @staticmethod
    def backward(ctx, dz2, _dm, _di):
        z1, g1, b1, mean1, invstd1, y1, w = ctx.saved_tensors
        dz2 = dz2.contiguous(memory_format=torch.channels_last)
        L = lib()
        dw, h = _wgrad_fork(_wgrad3x3_s2, dz2, y1, w) if ctx.needs_input_grad[6] else (None, None)
        sc, bi = ctx.aff1 or _affine(g1, b1, mean1, invstd1)
        if _own_dgb(g1, b1):   # bn1's parameter gradients from the sums' finalize launch
            dg1, db1 = torch.empty_like(g1), torch.empty_like(b1)
            dy1, s1, q1 = L.conv_gemm_s2dgrad(dz2, ctx.wr, _zero_row(dz2.device), z1, sc, bi,
                                              mean1, invstd1, dg1, db1)
        else:
            dy1, s1, q1 = L.conv_gemm_s2dgrad(dz2, ctx.wr, _zero_row(dz2.device), z1, sc, bi,
                                              mean1, invstd1)
            M = z1.numel() // z1.shape[1]
            _, _, _, dg1, db1 = L.bn_bwd_coeffs(s1, q1, g1, mean1, invstd1, M)
        dz1 = L.bn_bwd_apply(dy1, z1, g1, b1, mean1, invstd1, s1, q1)
        dw = _wgrad_join(dw, h)
        return dz1, dg1, db1, None, None, None, dw, None, None, None, None, None


def conv3x3_s2_ok(x: torch.Tensor, conv) -> bool:
    """Stride-2 padding-1 3x3 convs on NHWC bf16 GPU tensors with 64-multiple channels and an even
    input (every dx pixel then belongs to exactly one parity class)."""
    return (x.is_cuda and x.dtype == torch.bfloat16 and conv.weight.dtype == torch.bfloat16
            and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)
            and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0
            and conv.kernel_size == (3, 3) and conv.stride == (2, 2) and conv.padding == (1, 1)
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0)


def conv3x3_s2_bn_stats(x: torch.Tensor, conv, bn):
    """(z, (mean, invstd)) of a stride-2 ``conv(x)`` and bn's training statistics; callers check
    ``conv3x3_s2_ok``."""
    z, m, i = _Conv3x3S2BNStatsFn.apply(x, conv.weight, bn.running_mean, bn.running_var, bn.eps,
                                        bn.momentum, _fin_aff(bn))
    return z, (m, i)


def bnrelu_conv3x3_s2_bn_stats(z1: torch.Tensor, bn_a, stats_a, conv, bn):
    """``bnrelu_conv3x3_bn_stats`` for a stride-2 conv; callers check ``conv3x3_s2_ok`` on z1."""
    z, m, i = _BNReLUConv3x3S2BNStatsFn.apply(z1, bn_a.weight, bn_a.bias, stats_a[0], stats_a[1],
                                              bn_a.eps, conv.weight, bn.running_mean,
                                              bn.running_var, bn.eps, bn.momentum, _fin_aff(bn))
    return z, (m, i)


# PerfPolicy.bn1_dgrad_sums -- bn1 + ReLU -> 3x3 conv with bn1's backward sums in the data-gradient
# epilogue (off: bn_act + conv3x3_bn_stats, bn1's backward with its own reduction pass)


def bnrelu_conv3x3_bn_stats(z1: torch.Tensor, bn_a, stats_a, conv, bn):
    """(z, (mean, invstd)) of ``conv(relu(bn_a(z1)))`` (bn_a's batch statistics ``stats_a``) and
    bn's training statistics; callers check ``conv3x3_ok`` on z1 first."""
    z, m, i = _BNReLUConv3x3BNStatsFn.apply(z1, bn_a.weight, bn_a.bias, stats_a[0], stats_a[1],
                                            bn_a.eps, conv.weight, bn.running_mean, bn.running_var,
                                            bn.eps, bn.momentum, _fin_aff(bn))
    return z, (m, i)


def conv3x3_bn_stats(x: torch.Tensor, conv, bn):
    """(z, (mean, invstd)) of ``conv(x)`` and bn's training statistics (running stats updated),
    from one implicit-GEMM kernel; callers check ``conv3x3_ok`` first."""
    z, m, i = _Conv3x3BNStatsFn.apply(x, conv.weight, bn.running_mean, bn.running_var, bn.eps,
                                      bn.momentum, _fin_aff(bn))
    return z, (m, i)


def conv3x3_ok(x: torch.Tensor, conv) -> bool:
    """Stride-1 padding-1 3x3 convs on NHWC bf16 GPU tensors with 64-multiple channels."""
    return (x.is_cuda and x.dtype == torch.bfloat16 and conv.weight.dtype == torch.bfloat16
            and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)
            and conv.kernel_size == (3, 3) and conv.stride == (1, 1) and conv.padding == (1, 1)
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0)


def conv3x3(x: torch.Tensor, conv) -> torch.Tensor:
    """``conv(x)`` with the data gradient on the HIP implicit GEMM where eligible."""
    if conv3x3_ok(x, conv) and torch.is_grad_enabled():
        return _Conv3x3Fn.apply(x, conv.weight)
    return conv(x)


def conv1x1_bn_stats(x: torch.Tensor, conv, bn, stride: int = 1, dgrad_gemm: bool = False,
                     own_wgrad: bool = False, link=None):
    """(z, mean, invstd): 1x1 conv output and its training BN statistics (bn's running stats are
    updated). ``conv`` / ``bn``: nn.Conv2d-like (weight) and BatchNormAct2d modules."""
    return _Conv1x1BNStatsFn.apply(x, conv.weight, bn.running_mean, bn.running_var, stride,
                                   bn.eps, bn.momentum, dgrad_gemm, own_wgrad, link, _fin_aff(bn))


def bnrelu_conv1x1_bn_stats(z: torch.Tensor, bn_a, stats_a, conv, bn_b, dgrad_gemm: bool = False,
                            own_wgrad: bool = True):
    """(z3, mean3, invstd3) = conv(relu(bn_a(z))) + bn_b's statistics; bn_a's batch statistics
    ``stats_a`` = (mean, invstd) from ``bn_stats``."""
    mean, invstd = stats_a
    return _BNReLUConv1x1BNStatsFn.apply(z, bn_a.weight, bn_a.bias, mean, invstd, conv.weight,
                                         bn_b.running_mean, bn_b.running_var, bn_b.eps,
                                         bn_b.momentum, dgrad_gemm, own_wgrad)


def bn_stats(z: torch.Tensor, bn) -> Tuple[torch.Tensor, torch.Tensor]:
    """Training batch statistics (mean, invstd) of z; bn's running statistics are updated."""
    return tuple(lib().bn_stats(z, bn.running_mean, bn.running_var, bn.eps, bn.momentum))


def reference_conv1x1_bn(x: torch.Tensor, w: torch.Tensor, stride: int = 1,
                         pro: Optional[Tuple[torch.Tensor, torch.Tensor]] = None):
    """fp32 PyTorch oracle: (y, mean, biased var) of y = conv1x1(f(x)) (tests)."""
    xf = x.float()
    if pro is not None:
        xf = torch.relu(xf * pro[0].view(1, -1, 1, 1) + pro[1].view(1, -1, 1, 1))
        xf = xf.to(torch.bfloat16).float()   # the kernel stages the transformed input in bf16
    y = F.conv2d(xf, w.float(), stride=stride)
    yb = y.to(torch.bfloat16).float()
    return y, yb.mean((0, 2, 3)), yb.var((0, 2, 3), unbiased=False)
