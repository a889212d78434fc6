"""Transformer hot ops: fused cross-entropy, LayerNorm / RMSNorm (+ residual add), QKV split +
RoPE, SwiGLU and bias-gradient linear layers.

GPU bf16 tensors run the HIP kernels of ``csrc/kernels/transformer.hip``; every other input (CPU
tests, fp32) runs the equivalent PyTorch composition, which is also the numerics oracle of
``tests/test_transformer_ops_gpu.py``. Profiles that motivated each op are in
``profiles/r01_prof13_{bert,llama}_kernels.md`` (PyTorch's unfused paths: ~40 % of the Llama and
~25 % of the BERT step outside the GEMMs and attention).
"""
from __future__ import annotations

import math
import os
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..perf import policy as _P
from . import worker_grads as WG
from .bn import ResidualLink
from .native import lib


def _gpu_bf16(*ts: Optional[torch.Tensor]) -> bool:
    return all(t is None or (t.is_cuda and t.dtype == torch.bfloat16) for t in ts)


# ============================================================================ cross-entropy
# logits-bias gradients produced by the cross-entropy backward, keyed by the data pointer of the
# logits gradient it returned: the producing linear (``_LinearFn`` with a padded output) takes the
# fold instead of re-reading the R x V gradient for its column sums (same hand-off pattern as the
# ResidualLink sums of ops.conv)
_LOGIT_BIAS_PARTS = {}


def _row_strided(x: torch.Tensor) -> bool:
    """[R, V] with unit column stride and 16-B aligned padded rows (ld % 8 == 0, ld > V)."""
    return (x.dim() == 2 and x.stride(1) == 1 and x.stride(0) > x.shape[1]
            and x.stride(0) % 8 == 0)


class _CEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        lse, rows = lib().ce_fwd(logits, labels, ignore_index)
        # mean loss and the valid-label count in one launch (fixed-order fp64 sums; was five
        # ATen launches: ne, sum, clamp, cast, sum + divide)
        loss, count = lib().ce_mean(rows, labels, ignore_index)
        ctx.save_for_backward(logits, labels, lse, count)
        ctx.ignore = ignore_index
        return loss

    @staticmethod
    def backward(ctx, go):
        logits, labels, lse, count = ctx.saved_tensors
        # the kernels divide grad_output by the count themselves (no divide launch)
        go = go.float().reshape(1)
        if _row_strided(logits) and logits.shape[0] % 64 == 0:
            # padded logits of a biased linear: gradient rows with the same stride, and the bias
            # gradient's column partials from the same pass
            g, part = lib().ce_bwd_cs(logits, labels, lse, go, ctx.ignore, count)
            _LOGIT_BIAS_PARTS.clear()
            _LOGIT_BIAS_PARTS[g.data_ptr()] = (part, g.shape)
            return g, None, None
        return lib().ce_bwd(logits, labels, lse, go, ctx.ignore, count), None, None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor,
                  ignore_index: int = -100) -> torch.Tensor:
    """Mean cross-entropy of ``logits [..., V]`` against integer ``labels [...]``.

    bf16 GPU logits never get an fp32 copy: one read for the loss, one read + one bf16 write for
    the gradient (fp32 math inside). Row-strided logits (the padded output of a linear whose V is
    not a multiple of 8, ``linear``) are read in place, and their backward also emits the bias
    gradient's column sums. Other inputs use ``F.cross_entropy`` in fp32."""
    V = logits.shape[-1]
    if _gpu_bf16(logits) and labels.is_cuda:
        x = logits.reshape(-1, V)
        if not (x.is_contiguous() or _row_strided(x)):
            x = x.contiguous()
        if x.data_ptr() % 16:   # misaligned view (the kernel reads 16-B vectors)
            x = x.clone()
        return _CEFn.apply(x, labels.reshape(-1).long().contiguous(), int(ignore_index))
    return F.cross_entropy(logits.float().reshape(-1, V), labels.reshape(-1),
                           ignore_index=ignore_index)


def _take_bias_parts(dy2: torch.Tensor):
    """The cross-entropy's column partials for this logits gradient, if it left them."""
    hit = _LOGIT_BIAS_PARTS.pop(dy2.data_ptr(), None)
    if hit is not None and tuple(hit[1]) == tuple(dy2.shape):
        return hit[0]
    return None


# ============================================================================ norms
class _NormFn(torch.autograd.Function):
    """y = norm(x) (no residual)."""

    @staticmethod
    def forward(ctx, x, w, b, eps):
        y, _, mean, rstd = lib().norm_fwd(x, None, w, b, eps)
        ctx.save_for_backward(x, w, mean if b is not None else None, rstd)
        ctx.ln = b is not None
        ctx.params = (w, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, mean, rstd = ctx.saved_tensors
        seg = _norm_bwd_workers(ctx, dy, None, x, w, mean, rstd)
        if seg is not None:
            return seg, None, None, None
        dx, dw, db = lib().norm_bwd(dy, None, x, w, mean, rstd)
        return dx, dw, (db if ctx.ln else None), None


class _AddNormFn(torch.autograd.Function):
    """(s, y) = (x + r, norm(x + r)): the residual-stream update and the next sublayer's input in
    one pass. The backward adds the gradient of s (the stream's own consumers) to the norm's
    input gradient on the way out: d x = d r = ds + norm_bwd(dy)."""

    @staticmethod
    def forward(ctx, x, r, w, b, eps, x_link):
        y, s, mean, rstd = lib().norm_fwd(x, r, w, b, eps)
        ctx.save_for_backward(s, w, mean if b is not None else None, rstd)
        ctx.ln = b is not None
        ctx.params = (w, b)
        ctx.x_link = x_link
        # an unused s (post-LN BERT) must arrive as None, not as a zero-filled tensor that the
        # backward would then read
        ctx.set_materialize_grads(False)
        return s, y

    @staticmethod
    def backward(ctx, ds, dy):
        s, w, mean, rstd = ctx.saved_tensors
        if dy is None:
            return ds, ds, None, None, None, None
        seg = _norm_bwd_workers(ctx, dy, ds, s, w, mean, rstd)
        if seg is not None:
            dx, dw, db = seg, None, None
        else:
            dx, dw, db = lib().norm_bwd(dy, ds, s, w, mean, rstd)
        gx = dx
        link = ctx.x_link
        if link is not None and not link.closed and link.grad is None:
            # x's other consumer (the next sublayer's input GEMM, see linear(link=...)) runs its
            # backward later and absorbs this gradient in its beta = 1 epilogue
            link.grad = dx
            gx = None
        return gx, dx, dw, (db if ctx.ln else None), None, None


def _norm_bwd_workers(ctx, dy, ds, x, w, mean, rstd) -> Optional[torch.Tensor]:
    """Batched virtual workers (ops.worker_grads): dx, with worker v's dgamma / dbeta written to
    row v of the engine's gradient buffer; None when no per-worker destination is active."""
    wg = WG.current()
    pw, pb = ctx.params
    if wg is None or not wg.has(pw):
        return None
    V, D = wg.V, x.shape[-1]
    dwv, fw = wg.out(pw)
    dbv, fb = wg.out(pb) if ctx.ln else (None, True)
    if fw and fb:
        return lib().norm_bwd_seg(dy, ds, x, w, mean, rstd, V, dwv.view(V, D),
                                  dbv.view(V, D) if dbv is not None else None)
    tw = torch.empty(V, D, dtype=dwv.dtype, device=dwv.device)      # (second producer: add)
    tb = torch.empty_like(tw) if ctx.ln else None
    dx = lib().norm_bwd_seg(dy, ds, x, w, mean, rstd, V, tw, tb)
    (dwv.view(V, D).copy_ if fw else dwv.view(V, D).add_)(tw)
    if ctx.ln:
        (dbv.view(V, D).copy_ if fb else dbv.view(V, D).add_)(tb)
    return dx


def _norm_ref(x, w, b, eps):
    xf = x.float()
    if b is None:
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    else:
        y = F.layer_norm(xf, (x.shape[-1],), w.float(), b.float(), eps)
    return y.to(x.dtype)


def _norm_ok(x: torch.Tensor, D: int) -> bool:
    return D % 8 == 0 and D <= 4096 and x.is_contiguous() and x.data_ptr() % 16 == 0


def norm(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], eps: float) -> torch.Tensor:
    """LayerNorm (``b`` given) or RMSNorm (``b is None``) over the last dim."""
    if _gpu_bf16(x, w, b) and _norm_ok(x, x.shape[-1]):
        return _NormFn.apply(x, w, b, float(eps))
    return _norm_ref(x, w, b, eps)


def add_norm(x: torch.Tensor, r: Optional[torch.Tensor], w: torch.Tensor,
             b: Optional[torch.Tensor], eps: float,
             x_link: Optional[ResidualLink] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """(s, norm(s)) with s = x + r (r None: s = x). ``x_link``: x also feeds a ``linear(...,
    link=x_link)`` whose backward runs after this op's (x's gradient is then added inside that
    GEMM instead of by autograd)."""
    if r is None:
        return x, norm(x, w, b, eps)
    if _gpu_bf16(x, r, w, b) and _norm_ok(x, x.shape[-1]) and r.is_contiguous() \
            and r.data_ptr() % 16 == 0 and r.shape == x.shape:
        return _AddNormFn.apply(x, r, w, b, float(eps), x_link)
    s = x + r
    return s, _norm_ref(s, w, b, eps)


class RMSNorm(nn.Module):
    def __init__(self, d: int, eps: float = 1e-5):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(d))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return norm(x, self.weight, None, self.eps)


class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm whose bf16 GPU forward / backward run the fused HIP kernels."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return norm(x, self.weight, self.bias, self.eps)


# ============================================================================ BERT embedding
class _BertEmbedFn(torch.autograd.Function):
    """x = tok[ids] + pos[0:S] + typ[0] (segment 0 everywhere), the same three bf16 ops as the
    module composition. Its own backward so that batched virtual workers get per-worker
    embedding gradients (ops.worker_grads); otherwise the dense embedding backward of each
    table, as autograd would compute it."""

    @staticmethod
    def forward(ctx, ids, tok, pos, typ):
        S = ids.shape[1]
        x = F.embedding(ids, tok) + pos[:S][None] + typ[0]
        ctx.save_for_backward(ids)
        ctx.params = (tok, pos, typ)
        ctx.nums = (tok.shape[0], pos.shape[0])
        return x

    @staticmethod
    def backward(ctx, dx):
        (ids,) = ctx.saved_tensors
        tok, pos, typ = ctx.params
        nv, npos = ctx.nums
        B, S, D = dx.shape
        emb_bwd = torch.ops.aten.embedding_dense_backward

        def parts(d, i):
            gt = emb_bwd(d, i, nv, -1, False)
            gp = torch.zeros(npos, D, dtype=d.dtype, device=d.device)
            gp[:S] = d.sum(0)
            gy = torch.zeros(2, D, dtype=d.dtype, device=d.device)
            gy[0] = d.sum((0, 1))
            return gt, gp, gy

        wg = WG.current()
        if wg is not None and wg.has(tok):
            # all workers at once: token ids offset by v * vocab index one [V * vocab, D] table
            V = wg.V
            b = B // V
            off = (torch.arange(V, device=ids.device) * nv).view(V, 1, 1)
            gt = emb_bwd(dx, (ids.view(V, b, S) + off).view(B, S), V * nv, -1, False)
            gp = dx.view(V, b, S, D).sum(1)                   # [V, S, D]
            gy = dx.view(V, b * S, D).sum(1)                  # [V, D]
            for p, g, put in ((tok, gt.view(V, nv, D), None), (pos, gp, S), (typ, gy, 0)):
                dst, first = wg.out(p)
                if put is None:
                    (dst.copy_ if first else dst.add_)(g)
                elif put == 0:                                # segment 0 only
                    if first:
                        dst[:, 1:].zero_()
                        dst[:, 0].copy_(g)
                    else:
                        dst[:, 0].add_(g)
                else:                                         # positions [0, S)
                    if first:
                        dst[:, S:].zero_()
                        dst[:, :S].copy_(g)
                    else:
                        dst[:, :S].add_(g)
            return None, None, None, None
        gt, gp, gy = parts(dx, ids)
        return None, gt, gp, gy


def bert_embed(ids: torch.Tensor, tok: torch.Tensor, pos: torch.Tensor,
               typ: torch.Tensor) -> torch.Tensor:
    if _gpu_bf16(tok, pos, typ) and ids.is_cuda:
        return _BertEmbedFn.apply(ids, tok, pos, typ)
    S = ids.shape[1]
    return F.embedding(ids, tok) + pos[:S][None] + typ[0]


# ============================================================================ QKV split + RoPE
class _RopeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, H, KV, hd):
        ctx.set_materialize_grads(False)
        q, k, v = lib().rope_fwd(qkv, cos, sin, H, KV, hd)
        ctx.save_for_backward(cos, sin)
        ctx.has_rot = cos is not None
        ctx.shapes = (q.shape, k.shape)
        return q, k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        cos, sin = ctx.saved_tensors if ctx.has_rot else (None, None)
        qs, ks = ctx.shapes
        ref = next(t for t in (dq, dk, dv) if t is not None)
        dq = dq if dq is not None else ref.new_zeros(qs)
        dk = dk if dk is not None else ref.new_zeros(ks)
        dv = dv if dv is not None else ref.new_zeros(ks)
        return lib().rope_bwd(dq, dk, dv, cos, sin), None, None, None, None, None


def rope_tables(S: int, hd: int, theta: float, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """fp32 (cos, sin) [S, hd/2] for interleaved-pair rotary embeddings."""
    inv = 1.0 / (theta ** (torch.arange(0, hd, 2, device=device, dtype=torch.float32) / hd))
    f = torch.outer(torch.arange(S, device=device, dtype=torch.float32), inv)
    return f.cos().contiguous(), f.sin().contiguous()


def _rope_ref(x, cos, sin):
    """x [B, h, S, hd]; rotate pairs (x[2i], x[2i+1]) by (cos, sin)[s, i]."""
    xf = x.float()
    x1, x2 = xf[..., 0::2], xf[..., 1::2]
    c, s = cos[None, None], sin[None, None]
    return torch.stack((x1 * c - x2 * s, x1 * s + x2 * c), -1).flatten(-2).to(x.dtype)


def qkv_split(qkv: torch.Tensor, H: int, KV: int, hd: int, cos: Optional[torch.Tensor] = None,
              sin: Optional[torch.Tensor] = None):
    """Fused projection ``qkv [B, S, (H + 2 KV) hd]`` -> head-major contiguous ``q [B, H, S, hd]``,
    ``k, v [B, KV, S, hd]``, with RoPE on q / k when (cos, sin) fp32 [S, hd/2] are given."""
    B, S, _ = qkv.shape
    if _gpu_bf16(qkv) and hd % 8 == 0 and qkv.is_contiguous() and qkv.data_ptr() % 16 == 0:
        return _RopeFn.apply(qkv, cos, sin, H, KV, hd)
    x = qkv.view(B, S, H + 2 * KV, hd).transpose(1, 2)
    q, k, v = x[:, :H], x[:, H:H + KV], x[:, H + KV:]
    if cos is not None:
        q, k = _rope_ref(q, cos, sin), _rope_ref(k, cos, sin)
    return q.contiguous(), k.contiguous(), v.contiguous()


# ============================================================================ attention
class _AttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, H, scale):
        out, lse = lib().attn_fwd(qkv, H, scale)
        ctx.save_for_backward(qkv, out, lse)
        ctx.H, ctx.scale = H, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        return lib().attn_bwd(qkv, out, dout, lse, ctx.H, ctx.scale), None, None


def _attn_ok(qkv: torch.Tensor, H: int, hd: int) -> bool:
    S = qkv.shape[1]
    return (_gpu_bf16(qkv) and hd == 64 and S % 32 == 0 and 32 <= S <= 128
            and qkv.is_contiguous() and qkv.data_ptr() % 16 == 0 and _P().attn_kernel)


# PerfPolicy.attn_kernel: short-sequence MFMA attention for BERT-shaped problems (off: SDPA)


def fused_qkv_attention(qkv: torch.Tensor, H: int, hd: int) -> torch.Tensor:
    """Non-causal multi-head attention straight from the fused projection ``qkv [B, S, 3 H hd]``
    to ``[B, S, H hd]`` (the output projection's input layout). S <= 128, hd = 64 bf16 GPU
    tensors run csrc/kernels/attention.hip (one workgroup per (batch, head), MFMA, exact
    softmax); anything else splits the heads and runs SDPA."""
    B, S, _ = qkv.shape
    if _attn_ok(qkv, H, hd):
        return _AttnFn.apply(qkv, H, 1.0 / math.sqrt(hd))
    q, k, v = qkv_split(qkv, H, H, hd)
    return F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, S, H * hd)


# ============================================================================ flash attention
def _flash_ok(*ts: torch.Tensor) -> bool:
    return (_P().flash_attn and _gpu_bf16(*ts)
            and all(t.is_contiguous() and t.data_ptr() % 16 == 0 for t in ts))


class _FlashFn(torch.autograd.Function):
    """softmax(q k^T scale [+ causal mask]) v on csrc/kernels/flash_attn.hip: q [B, H, S, 128],
    k / v [B, KV, S, 128] -> o [B, S, H * 128]. The backward's per-query-head dk / dv are summed
    over each kv head's group here (the fused QKV path, ``_RopeFlashFn``, sums them inside the RoPE
    backward kernel instead)."""

    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        o, lse = lib().flash_fwd(q, k, v, causal, scale)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        dq, dkh, dvh = lib().flash_bwd(q, k, v, o, do, lse, ctx.causal, ctx.scale)
        B, H, S, D = q.shape
        KV = k.shape[1]
        if H != KV:
            dkh = dkh.view(B, KV, H // KV, S, D).float().sum(2).to(q.dtype)
            dvh = dvh.view(B, KV, H // KV, S, D).float().sum(2).to(q.dtype)
        return dq, dkh, dvh, None, None


def _sdpa_rows(q, k, v, causal: bool, scale: float) -> torch.Tensor:
    """Reference composition of flash_attention (any device / dtype): [B, S, H * hd]."""
    B, H, S, hd = q.shape
    o = F.scaled_dot_product_attention(q, k, v, is_causal=causal, scale=scale,
                                       enable_gqa=H != k.shape[1])
    return o.transpose(1, 2).reshape(B, S, H * hd)


def flash_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True,
                    scale: Optional[float] = None) -> torch.Tensor:
    """Multi-head attention with grouped-query heads (H % KV == 0): q [B, H, S, hd], k / v
    [B, KV, S, hd] -> [B, S, H * hd] (the output projection's input rows). bf16 GPU tensors with
    hd = 128 run the flash kernels of csrc/kernels/flash_attn.hip (forward and backward);
    anything else runs SDPA."""
    hd = q.shape[-1]
    scale = float(scale) if scale is not None else 1.0 / math.sqrt(hd)
    if hd == 128 and _flash_ok(q, k, v):
        return _FlashFn.apply(q, k, v, bool(causal), scale)
    return _sdpa_rows(q, k, v, causal, scale)


class _RopeFlashFn(torch.autograd.Function):
    """QKV split + RoPE + flash attention from the fused projection ``qkv [B, S, (H + 2 KV) 128]``
    to ``o [B, S, H 128]``. Backward: the flash backward, then ONE RoPE-backward pass that also
    sums the per-query-head dk / dv of each kv head's group (transformer.hip rope_bwd, grp) and
    writes dqkv in the fused layout."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, H, KV, causal, scale):
        q, k, v = lib().rope_fwd(qkv, cos, sin, H, KV, 128)
        o, lse = lib().flash_fwd(q, k, v, causal, scale)
        ctx.save_for_backward(q, k, v, o, lse, cos, sin)
        ctx.cfg = (H, KV, causal, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, cos, sin = ctx.saved_tensors
        H, KV, causal, scale = ctx.cfg
        dq, dkh, dvh = lib().flash_bwd(q, k, v, o, do, lse, causal, scale)
        dqkv = lib().rope_bwd(dq, dkh, dvh, cos, sin, H // KV)
        return dqkv, None, None, None, None, None, None


def qkv_attention(qkv: torch.Tensor, H: int, KV: int, hd: int,
                  cos: Optional[torch.Tensor] = None, sin: Optional[torch.Tensor] = None,
                  causal: bool = True) -> torch.Tensor:
    """Attention straight from the fused projection ``qkv [B, S, (H + 2 KV) hd]`` (RoPE on q / k
    when cos / sin are given) to ``[B, S, H hd]``. bf16 GPU tensors with hd = 128 run
    ``_RopeFlashFn`` (own kernels end to end); otherwise qkv_split + SDPA."""
    scale = 1.0 / math.sqrt(hd)
    if hd == 128 and _flash_ok(qkv) and (cos is None or (cos.is_cuda and sin.is_cuda)):
        return _RopeFlashFn.apply(qkv, cos, sin, H, KV, bool(causal), scale)
    q, k, v = qkv_split(qkv, H, KV, hd, cos, sin)
    return _sdpa_rows(q, k, v, causal, scale)


# ============================================================================ SwiGLU
class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h):
        ctx.save_for_backward(h)
        return lib().swiglu_fwd(h)

    @staticmethod
    def backward(ctx, dy):
        (h,) = ctx.saved_tensors
        return lib().swiglu_bwd(dy, h)


def swiglu(h: torch.Tensor) -> torch.Tensor:
    """silu(a) * b for h = [a | b] along the last dim."""
    F2 = h.shape[-1]
    if _gpu_bf16(h) and F2 % 16 == 0 and h.is_contiguous() and h.data_ptr() % 16 == 0:
        return _SwiGLUFn.apply(h)
    a, b = h.chunk(2, -1)
    return F.silu(a) * b


# ============================================================================ linear (bias grad)
def _al16(*ts: Optional[torch.Tensor]) -> bool:
    """Contiguous and 16-B aligned (gemm.hip reads 16-B vectors: a contiguous view at an odd
    element offset would fail the launch instead of falling back)."""
    return all(t is None or (t.is_contiguous() and t.data_ptr() % 16 == 0) for t in ts)


def _own_gemm(M: int, N: int, K: int) -> bool:
    """Own NT GEMM (gemm_nt, ep 0) for a bf16 GEMM of this shape: gemm.hip's 256 x 256 tiles when
    they fill the chip (>= 128 tiles), else gemm128.hip's 128 x 128 tiles (PerfPolicy.own_gemm128;
    at the BERT per-rank shapes 1.15-1.8x hipBLASLt, profiles/r05_05/gemm.jsonl)."""
    if not _P().own_gemm:
        return False
    try:
        pick = int(lib().gemm_nt_pick(M, N, K))
    except Exception:
        return False
    return pick == 256 or (pick == 128 and _P().own_gemm128)


def _linear_wgrad(gout: torch.Tensor, gin: torch.Tensor) -> torch.Tensor:
    """dW [N, K] = gout^T gin over T token rows (gout [T, N], gin [T, K]). PerfPolicy.own_linear_wgrad:
    on the 1x1-conv weight-gradient kernel (wgrad1x1.hip: row-major [T, C] activations are NHWC
    [T, C, 1, 1]; split-K over the rows, fixed-order fold), else hipBLASLt. Up to BERT-base sizes
    (N K <= 4 M): at T = 8192 the kernel matches hipBLASLt on 2304 / 3072-wide shapes and is 1.5x
    faster on 768 x 768 (bench/linear_wgrad.py), and the BERT V = 1 x 64 step drops 13.55 -> 12.94
    ms (profiles/r04_38/). Llama-3-8B weights (one split on the LDS-DMA kernel, dW written
    directly) run 0.89-1.12 PFLOP/s there vs 1.0-1.39 for hipBLASLt NT on transposed operands,
    transposes included (profiles/r05_33/llama_wgrad.jsonl): they stay on the NT path."""
    T, N = gout.shape
    K = gin.shape[-1]
    if (_P().own_linear_wgrad and gout.is_cuda and gout.dtype == torch.bfloat16
            and gin.dtype == torch.bfloat16 and N % 128 == 0 and K % 128 == 0
            and N * K <= 4 * 1024 * 1024
            and gout.is_contiguous() and gin.is_contiguous()):
        return lib().wgrad1x1(gout.view(T, 1, 1, N).permute(0, 3, 1, 2),
                              gin.view(T, 1, 1, K).permute(0, 3, 1, 2), torch.bfloat16).view(N, K)
    return gout.t() @ gin


# persistent zero-padded copies of logits-head weights / biases (padded_logits), held ON the weight
# parameter itself (attribute ``_cml_pad``, keyed by the bias's identity): released together with
# the parameter, never matched by a new tensor that reuses an id; refreshed in place each forward
# (rows N .. Np stay zero), so the padded path costs one weight copy instead of an allocation +
# zero-fill + copy per step


def _padded_wb(w: torch.Tensor, b: torch.Tensor, Np: int):
    hit = getattr(w, "_cml_pad", None)
    if (hit is None or hit[2] is not b or hit[0].shape[0] != Np or hit[0].device != w.device
            or hit[0].dtype != w.dtype):
        hit = (w.new_zeros(Np, w.shape[1]), b.new_zeros(Np), b)
        w._cml_pad = hit
    wp, bp = hit[0], hit[1]
    N = w.shape[0]
    wp[:N].copy_(w)
    bp[:N].copy_(b)
    return wp, bp


class _LinearFn(torch.autograd.Function):
    """y = x W^T + b with the bias gradient from the column-sum kernel (PyTorch's generic column
    reduction runs these at ~0.4 TB/s: 7 % of the BERT step in profiles/r01_prof13)."""

    @staticmethod
    def forward(ctx, x, w, b, link, pad_logits=False):
        ctx.save_for_backward(x, w)
        ctx.link = link
        ctx.params = (w, b)
        x2 = x.reshape(-1, x.shape[-1])
        N = w.shape[0]
        if _own_gemm(x2.shape[0], N, w.shape[1]) and _al16(x2, w, b):
            return lib().gemm_nt(x2, w, 0, bias=b).view(*x.shape[:-1], N)
        if pad_logits and b is not None and N % 8 and x2.shape[0] % 64 == 0:
            # logits feeding the cross-entropy (BertMLM's head, V = 30522, not a multiple of 8):
            # the GEMM writes rows padded to Np (zero weight rows / bias), the output is the
            # [.., N] view -- 16-B aligned rows for the cross-entropy kernels, whose backward then
            # also emits the bias gradient
            Np = (N + 7) // 8 * 8
            wp, bp = _padded_wb(w, b, Np)
            y = F.linear(x2, wp, bp)
            return y.view(*x.shape[:-1], Np)[..., :N]
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        return _linear_grads(ctx, dy.reshape(-1, dy.shape[-1]), x, w) + (None, None)


def _linear_grads(ctx, dy2: torch.Tensor, x: torch.Tensor, w: torch.Tensor):
    """(dx, dw, db) of y = x W^T + b from the output gradient rows dy2 [M, N] (ctx: needs_input_grad
    over (x, w, b), ``link``, ``params`` = (w, b) modules' tensors). Batched virtual workers write
    per-worker dW / db straight into their gradient rows and return dw = db = None."""
    dx = dw = db = None
    # bias-gradient column partials left by the cross-entropy backward (padded logits)
    parts = _take_bias_parts(dy2) if ctx.needs_input_grad[2] and dy2.is_cuda else None
    if ctx.needs_input_grad[0]:
        g = ctx.link.take() if ctx.link is not None else None
        K = x.shape[-1]
        own = _own_gemm(dy2.shape[0], K, w.shape[0]) and _al16(dy2)
        if own and (g is None or (_al16(g) and g.shape == x.shape)):
            # data gradient on gemm.hip against the transposed weight, the parked residual
            # gradient added in the epilogue (in place)
            wt = lib().transpose_bf16(w)
            if g is not None:
                g2 = g.view(-1, K)
                dx = lib().gemm_nt(dy2, wt, 0, out=g2, cin=g2).view(x.shape)
            else:
                dx = lib().gemm_nt(dy2, wt, 0).view(x.shape)
        elif g is not None and g.is_contiguous() and g.shape == x.shape:
            dx = g.view(-1, x.shape[-1]).addmm_(dy2, w).view(x.shape)   # beta = 1 epilogue
        elif g is not None:
            dx = (g.reshape(-1, x.shape[-1]) + dy2 @ w).view(x.shape)
        else:
            dx = (dy2 @ w).view(x.shape)
    wg = WG.current()
    pw, pb = ctx.params
    if wg is not None and (wg.has(pw) or (pb is not None and wg.has(pb))):
        # batched virtual workers: per-worker dW / db straight into the gradient rows
        V, N, K = wg.V, dy2.shape[-1], x.shape[-1]
        T = dy2.shape[0] // V
        if ctx.needs_input_grad[1] and wg.has(pw):
            dst, first = wg.out(pw)
            if V == 1 and _P().own_linear_wgrad:
                d = _linear_wgrad(dy2, x.reshape(T, K))
                (dst.view(N, K).copy_ if first else dst.view(N, K).add_)(d)
            elif first:
                torch.bmm(dy2.view(V, T, N).transpose(1, 2), x.reshape(V, T, K),
                          out=dst.view(V, N, K))
            else:
                dst.view(V, N, K).baddbmm_(dy2.view(V, T, N).transpose(1, 2), x.reshape(V, T, K))
        if ctx.needs_input_grad[2] and pb is not None and wg.has(pb):
            dst, first = wg.out(pb)
            if parts is not None and T % 64 == 0:
                tgt = dst.view(V, N) if first else torch.empty(V, N, dtype=dst.dtype,
                                                               device=dst.device)
                lib().ce_part_fold(parts, N, V, tgt)
                if not first:
                    dst.view(V, N).add_(tgt)
            elif first and N % 8 == 0 and T % 32 == 0 and dy2.is_cuda and dy2.is_contiguous():
                lib().colsum_seg(dy2, V, dst.view(V, N))
            else:
                g = dy2.view(V, T, N).sum(1)
                (dst.copy_ if first else dst.add_)(g)
        return dx, None, None
    if ctx.needs_input_grad[1]:
        dw = _linear_wgrad(dy2, x.reshape(-1, x.shape[-1]))
    if ctx.needs_input_grad[2]:
        if parts is not None:
            db = torch.empty(1, dy2.shape[-1], dtype=dy2.dtype, device=dy2.device)
            lib().ce_part_fold(parts, dy2.shape[-1], 1, db)
            db = db.view(-1)
        else:
            db = lib().colsum(dy2) if (dy2.shape[-1] % 8 == 0 and dy2.is_contiguous()) \
                else dy2.sum(0)
    return dx, dw, db


class _LinearGeluFn(torch.autograd.Function):
    """a = gelu(x W^T + b) (erf GELU) on gemm.hip with bias + GELU in the epilogue (h kept for the
    backward), backward dh = da * gelu'(h) in one elementwise pass (``gelu_bwd``), then the linear's
    gradients as ``_LinearFn`` (BERT's MLM-head transform; the PyTorch GELU kernels it replaces:
    profiles/r04_06/bert_kernels.md)."""

    @staticmethod
    def forward(ctx, x, w, b):
        x2 = x.reshape(-1, x.shape[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        h = torch.empty(x2.shape[0], w.shape[0], dtype=x.dtype, device=x.device)
        a = lib().gemm_nt(x2, w, 1, bias=b, aux=h)
        ctx.save_for_backward(x2, w, h)
        ctx.link = None
        ctx.params = (w, b)
        ctx.xshape = x.shape
        return a.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, da):
        x2, w, h = ctx.saved_tensors
        dh = lib().gelu_bwd(da.reshape(-1, da.shape[-1]).contiguous(), h)
        dx, dw, db = _linear_grads(ctx, dh, x2, w)
        return (dx.view(ctx.xshape) if dx is not None else None), dw, db


def linear_gelu(x: torch.Tensor, lin: nn.Linear) -> torch.Tensor:
    """gelu(lin(x)) (erf GELU); gemm.hip-eligible bf16 GPU shapes run the fused-epilogue path."""
    w, b = lin.weight, lin.bias
    M = x.numel() // x.shape[-1]
    if (_P().fused_ffn and _gpu_bf16(x, w, b) and b is not None and _al16(w, b)
            and (not x.is_contiguous() or x.data_ptr() % 16 == 0)
            and _gemm_ok(M, w.shape[0], w.shape[1])):
        return _LinearGeluFn.apply(x, w, b)
    return F.gelu(lin(x))


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None,
           link: Optional[ResidualLink] = None, logits: bool = False) -> torch.Tensor:
    """``link``: a ResidualLink on which a later-in-forward op (``add_norm(x_link=...)``) parks
    another gradient of x; this GEMM's data-gradient absorbs it (beta = 1). ``logits``: the
    output only feeds ``cross_entropy`` -- with N % 8 != 0 it may come back as a view of
    16-B aligned padded rows (PerfPolicy.padded_logits); other callers always get a plain
    contiguous [.., N] tensor."""
    wg = WG.current()
    pad = logits and _P().padded_logits
    if _gpu_bf16(x, w, b) and ((b is not None and (w.shape[0] % 8 == 0 or pad))
                               or (wg is not None and wg.has(w))):
        return _LinearFn.apply(x, w, b, link, pad)
    return F.linear(x, w, b)


# own data gradient (gemm.hip against the transposed weight) for bias-free linears up to this
# many weight elements. With gemm.hip's grouped tile order (round 6) its data gradients run
# 1.05-1.31x hipBLASLt on every Llama-3-8B weight before the transpose: wqkv / wo / w2 (<= 64 M
# elements) still win with it, the w13 / output-head ones tie (profiles/r06_16/llama_gemm.jsonl)
_NB_OWN_DGRAD_MAX = 64 * 1024 * 1024
# own forward (gemm.hip NT, x W^T as stored) for weights up to this many elements with K up to
# _NB_OWN_FWD_KMAX: Llama-3-8B wqkv 1.37 vs 1.31 PFLOP/s for hipBLASLt, wo 1.35 vs 1.40, w13 1.434
# vs 1.433; the long-K w2 (K 14336: 1.46 vs 1.51) and the output head (1.44 vs 1.47) stay on
# hipBLASLt (profiles/r06_16/llama_gemm.jsonl)
_NB_OWN_FWD_MAX = int(os.environ.get("CML_NB_OWN_FWD_MAX", str(128 * 1024 * 1024)))
_NB_OWN_FWD_KMAX = 8192


class _LinearNBFn(torch.autograd.Function):
    """y = x W^T without bias (Llama's projections): forward on gemm.hip for weights up to
    _NB_OWN_FWD_MAX elements and K <= _NB_OWN_FWD_KMAX, else hipBLASLt (NT, its best layout).
    Backward: dx = dy W on gemm.hip for weights up to _NB_OWN_DGRAD_MAX elements, else hipBLASLt;
    dW = dy^T x as an NT GEMM on transposed operands -- (dy^T) (x^T)^T, two bandwidth-bound
    transposes + hipBLASLt NT at 1.3-1.57 PFLOP/s instead of its dy^T x kernels at 0.9-1.15
    (PerfPolicy.nt_wgrad; -0.5 ms per Llama-3-8B layer, profiles/r05_06/llama_gemm.jsonl)."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        ctx.param = w   # the Parameter itself (its id keys the direct-gradient destination)
        N, K = w.shape
        if x.is_contiguous() and w.numel() <= _NB_OWN_FWD_MAX and K <= _NB_OWN_FWD_KMAX:
            x2 = x.view(-1, K)
            if _own_gemm(x2.shape[0], N, K) and lib().gemm_nt_pick(x2.shape[0], N, K) == 256 \
                    and _al16(x2, w):
                return lib().gemm_nt(x2, w, 0).view(*x.shape[:-1], N)
        return F.linear(x, w)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        N, K = w.shape
        x2 = x.reshape(-1, K)
        dy2 = dy.reshape(-1, N)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        M = dy2.shape[0]
        L = lib()
        dx = dw = None
        if ctx.needs_input_grad[0]:
            if w.numel() <= _NB_OWN_DGRAD_MAX and _own_gemm(M, K, N) and _al16(dy2):
                dx = L.gemm_nt(dy2, L.transpose_bf16(w), 0)
            else:
                dx = dy2 @ w
            dx = dx.view(x.shape)
        if ctx.needs_input_grad[1]:
            wg = WG.current()
            dst, first = (None, True)
            if wg is not None and wg.V == 1 and wg.has(ctx.param):
                # direct gradient (engine TopologyConfig.direct_grads): written into the flat
                # gradient row, no autograd tensor and no capture copy
                dst, first = wg.out(ctx.param)
                dst = dst.view(N, K)
            if _P().nt_wgrad:
                a, b = L.transpose_bf16(dy2), L.transpose_bf16(x2).t()
            else:
                a, b = dy2.t(), x2
            if dst is None:
                dw = torch.matmul(a, b)
            elif first:
                torch.matmul(a, b, out=dst)
            else:
                dst.add_(torch.matmul(a, b))
        ctx.param = None
        return dx, dw


def linear_nb(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """Bias-free linear (``_LinearNBFn`` on bf16 GPU tensors, F.linear otherwise). Under a
    one-worker gradient destination (direct gradients) the weight gradient goes to the flat row;
    batched workers (V > 1) take ``linear`` (per-worker strided GEMMs)."""
    wg = WG.current()
    if _gpu_bf16(x, w) and (wg is None or wg.V == 1):
        return _LinearNBFn.apply(x, w)
    if wg is not None and wg.has(w):
        return linear(x, w, None)
    return F.linear(x, w)


class LinearNB(nn.Linear):
    """Bias-free nn.Linear whose bf16 GPU backward runs ``_LinearNBFn``."""

    def __init__(self, in_features: int, out_features: int):
        super().__init__(in_features, out_features, bias=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return linear_nb(x, self.weight)


class Linear(nn.Linear):
    """nn.Linear with the fused bias-gradient backward on bf16 GPU tensors."""

    def forward(self, x: torch.Tensor, link: Optional[ResidualLink] = None) -> torch.Tensor:
        return linear(x, self.weight, self.bias, link)


# ============================================================================ fused GELU FFN
def _gemm_ok(M: int, N: int, K: int) -> bool:
    try:
        return bool(lib().gemm_nt_ok(M, N, K))
    except Exception:
        return False


def _bias_grad_rows(b: torch.Tensor, V: int):
    """(destination [V, N] of the bias gradient, scatter-back or None): the engine's per-worker
    rows when batched workers own b, else a fresh [1, N] tensor."""
    wg = WG.current()
    if wg is not None and wg.has(b):
        dst, first = wg.out(b)
        dst = dst.view(V, -1)
        if first:
            return dst, None
        tmp = torch.empty_like(dst)
        return tmp, (lambda: dst.add_(tmp))
    return torch.empty(1, b.shape[0], dtype=b.dtype, device=b.device), None


class _FFNGeluFn(torch.autograd.Function):
    """y = fc2(gelu(fc1(x))) with the elementwise work in GEMM epilogues (csrc/kernels/gemm.hip):

    forward   fc1 on gemm.hip, epilogue h = x W1^T + b1 (kept for the backward) and a = gelu(h);
              fc2 = a W2^T + b2 (hipBLASLt)
    backward  dh = (dy W2) * gelu'(h) as ONE gemm.hip launch (dy against the transposed W2), with
              the fc1 bias gradient as column sums in the same epilogue (per worker segment for
              batched virtual workers); weight gradients and dx on hipBLASLt
    The unfused composition rounds h, a, da and dh to bf16 at the same points."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, link):
        x2 = x.reshape(-1, x.shape[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        M, F1 = x2.shape[0], w1.shape[0]
        h = torch.empty(M, F1, dtype=x.dtype, device=x.device)
        a = lib().gemm_nt(x2, w1, 1, bias=b1, aux=h)
        y = (lib().gemm_nt(a, w2, 0, bias=b2) if _own_gemm(M, w2.shape[0], F1) and _al16(w2, b2)
             else F.linear(a, w2, b2))
        ctx.save_for_backward(x2, w1, w2, h, a)
        ctx.link = link
        ctx.params = (w1, b1, w2, b2)
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w1, w2, h, a = ctx.saved_tensors
        pw1, pb1, pw2, pb2 = ctx.params
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        wg = WG.current()
        # per-worker fc1 bias-gradient rows only when the batched-workers object owns b1 (else
        # one [1, N] total, returned to autograd below)
        V = wg.V if wg is not None and wg.has(pb1) else 1
        cs, post = _bias_grad_rows(pb1, V)
        dh = lib().gemm_nt(dy2, lib().transpose_bf16(w2), 2, aux=h, colsum_out=cs)
        if post is not None:
            post()
        dx = None
        if ctx.needs_input_grad[0]:
            g = ctx.link.take() if ctx.link is not None else None
            K = x2.shape[-1]
            if _own_gemm(dh.shape[0], K, dh.shape[1]) and (
                    g is None or (_al16(g) and g.shape == ctx.xshape)):
                w1t = lib().transpose_bf16(w1)
                if g is not None:
                    g2 = g.view(-1, K)
                    dx = lib().gemm_nt(dh, w1t, 0, out=g2, cin=g2).view(ctx.xshape)
                else:
                    dx = lib().gemm_nt(dh, w1t, 0).view(ctx.xshape)
            elif g is not None and g.is_contiguous() and g.shape == ctx.xshape:
                dx = g.view(-1, x2.shape[-1]).addmm_(dh, w1).view(ctx.xshape)
            elif g is not None:
                dx = (g.reshape(-1, x2.shape[-1]) + dh @ w1).view(ctx.xshape)
            else:
                dx = (dh @ w1).view(ctx.xshape)
        if wg is not None and (wg.has(pw1) or wg.has(pw2)):
            T = dy2.shape[0] // wg.V
            for pw, gout, gin in ((pw1, dh, x2), (pw2, dy2, a)):
                dst, first = wg.out(pw)
                if wg.V == 1 and _P().own_linear_wgrad:
                    d = _linear_wgrad(gout, gin)
                    (dst.view_as(d).copy_ if first else dst.view_as(d).add_)(d)
                    continue
                A = gout.view(wg.V, T, -1).transpose(1, 2)
                Bm = gin.view(wg.V, T, -1)
                if first:
                    torch.bmm(A, Bm, out=dst.view(wg.V, pw.shape[0], pw.shape[1]))
                else:
                    dst.view(wg.V, pw.shape[0], pw.shape[1]).baddbmm_(A, Bm)
            db2 = None
            if wg.has(pb2):
                dst, first = wg.out(pb2)
                if first:
                    lib().colsum_seg(dy2, wg.V, dst.view(wg.V, -1))
                else:
                    dst.view(wg.V, -1).add_(dy2.view(wg.V, T, -1).sum(1))
            elif ctx.needs_input_grad[4]:
                db2 = lib().colsum(dy2)
            # biases the workers object does not own still get their (summed) gradients
            db1 = cs.view(-1) if (not wg.has(pb1) and ctx.needs_input_grad[2]) else None
            return dx, None, db1, None, db2, None
        dw1 = _linear_wgrad(dh, x2) if ctx.needs_input_grad[1] else None
        db1 = cs.view(-1) if ctx.needs_input_grad[2] else None
        dw2 = _linear_wgrad(dy2, a) if ctx.needs_input_grad[3] else None
        db2 = lib().colsum(dy2) if ctx.needs_input_grad[4] else None
        return dx, dw1, db1, dw2, db2, None


def ffn_gelu(x: torch.Tensor, fc1: nn.Linear, fc2: nn.Linear,
             link: Optional[ResidualLink] = None) -> torch.Tensor:
    """fc2(gelu(fc1(x))) (erf GELU). bf16 GPU tensors of gemm.hip-eligible shapes (tokens and FFN
    width multiples of 256) run the fused epilogue path; everything else the composition."""
    w1, b1, w2, b2 = fc1.weight, fc1.bias, fc2.weight, fc2.bias
    M = x.numel() // x.shape[-1]
    wg = WG.current()
    ok = (_P().fused_ffn and _gpu_bf16(x, w1, b1, w2, b2) and b1 is not None
          and b2 is not None and _al16(w1, b1, w2, b2)
          and (not x.is_contiguous() or x.data_ptr() % 16 == 0)
          and _gemm_ok(M, w1.shape[0], w1.shape[1])
          and _gemm_ok(M, w1.shape[0], w2.shape[0]) and w2.shape[0] % 8 == 0
          and (wg is None or M % (128 * wg.V) == 0))
    if ok:
        return _FFNGeluFn.apply(x, w1, b1, w2, b2, link)
    return fc2(F.gelu(fc1(x, link)))
