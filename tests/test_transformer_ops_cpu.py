"""CPU reference paths of ops/transformer.py (the numerics oracles of the HIP kernels) against
independent PyTorch formulations, and the restructured BERT / Llama blocks (fused QKV and gate-up
projections, residual adds fused into the next norm) against a plain layer-by-layer
re-implementation with the same weights."""
import math

import torch
import torch.nn.functional as F

from consensusml_amd.models import transformer as MT
from consensusml_amd.ops import transformer as T


def test_cross_entropy_cpu_matches_torch():
    torch.manual_seed(0)
    x = torch.randn(6, 11)
    y = torch.randint(0, 11, (6,))
    y[2] = -100
    torch.testing.assert_close(T.cross_entropy(x, y), F.cross_entropy(x, y, ignore_index=-100))


def test_add_norm_cpu():
    torch.manual_seed(1)
    x, r = torch.randn(5, 16), torch.randn(5, 16)
    w, b = torch.rand(16) + 0.5, torch.randn(16)
    s, y = T.add_norm(x, r, w, b, 1e-5)
    torch.testing.assert_close(s, x + r)
    torch.testing.assert_close(y, F.layer_norm(x + r, (16,), w, b, 1e-5))
    s, y = T.add_norm(x, None, w, None, 1e-5)
    assert s is x
    torch.testing.assert_close(y, x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * w)


def test_qkv_split_rope_cpu():
    torch.manual_seed(2)
    B, S, H, KV, hd = 2, 5, 4, 2, 8
    qkv = torch.randn(B, S, (H + 2 * KV) * hd)
    cos, sin = T.rope_tables(S, hd, 10000.0, "cpu")
    q, k, v = T.qkv_split(qkv, H, KV, hd, cos, sin)
    # complex-number formulation of interleaved RoPE
    def rope_c(t):
        tc = torch.view_as_complex(t.reshape(*t.shape[:-1], hd // 2, 2).contiguous())
        ang = torch.polar(torch.ones_like(cos), torch.atan2(sin, cos))
        return torch.view_as_real(tc * ang[None, None]).flatten(-2)
    x = qkv.view(B, S, H + 2 * KV, hd).transpose(1, 2)
    torch.testing.assert_close(q, rope_c(x[:, :H]), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(k, rope_c(x[:, H:H + KV]), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(v, x[:, H + KV:])
    assert q.is_contiguous() and k.is_contiguous() and v.is_contiguous()


def test_swiglu_and_linear_cpu():
    torch.manual_seed(3)
    h = torch.randn(4, 32)
    torch.testing.assert_close(T.swiglu(h), F.silu(h[:, :16]) * h[:, 16:])
    x, w, b = torch.randn(3, 8), torch.randn(6, 8), torch.randn(6)
    torch.testing.assert_close(T.linear(x, w, b), x @ w.t() + b)


def _bert_layer_plain(l, x):
    B, S, D = x.shape
    q, k, v = l.qkv(x).view(B, S, 3, l.h, D // l.h).permute(2, 0, 3, 1, 4)
    a = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, S, D)
    x = F.layer_norm(x + l.o(a), (D,), l.ln1.weight, l.ln1.bias, l.ln1.eps)
    return F.layer_norm(x + l.fc2(F.gelu(l.fc1(x))), (D,), l.ln2.weight, l.ln2.bias, l.ln2.eps)


def test_bert_layer_matches_plain():
    torch.manual_seed(4)
    m = MT.bert_tiny()
    x = torch.randn(2, 7, m.c.d)
    for l in m.layers:
        torch.testing.assert_close(l(x), _bert_layer_plain(l, x), rtol=1e-5, atol=1e-5)


def test_llama_matches_plain():
    """Fused projections + residual-fused norms == the textbook pre-norm Llama block."""
    torch.manual_seed(5)
    m = MT.llama_tiny()
    c = m.c
    ids = torch.randint(0, c.vocab, (2, 9))
    hd = c.d // c.heads
    cos, sin = T.rope_tables(9, hd, c.rope_theta, "cpu")

    def rms(x, w):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + c.eps) * w

    def rope(t):
        t1, t2 = t[..., 0::2], t[..., 1::2]
        return torch.stack((t1 * cos - t2 * sin, t1 * sin + t2 * cos), -1).flatten(-2)

    x = m.tok(ids)
    B, S, D = x.shape
    nq, nk = c.heads * hd, c.kv_heads * hd
    for l in m.layers:
        h = rms(x, l.n1.weight)
        wq, wk, wv = l.wqkv.weight.split([nq, nk, nk])
        q = rope((h @ wq.t()).view(B, S, c.heads, hd).transpose(1, 2))
        k = rope((h @ wk.t()).view(B, S, c.kv_heads, hd).transpose(1, 2))
        v = (h @ wv.t()).view(B, S, c.kv_heads, hd).transpose(1, 2)
        rep = c.heads // c.kv_heads
        k, v = k.repeat_interleave(rep, 1), v.repeat_interleave(rep, 1)
        att = (q @ k.transpose(-1, -2)) / math.sqrt(hd)
        att = att.masked_fill(torch.ones(S, S, dtype=torch.bool).triu(1), float("-inf"))
        a = (att.softmax(-1) @ v).transpose(1, 2).reshape(B, S, D)
        x = x + a @ l.wo.weight.t()
        h = rms(x, l.n2.weight)
        w1, w3 = l.w13.weight.chunk(2, 0)
        x = x + (F.silu(h @ w1.t()) * (h @ w3.t())) @ l.w2.weight.t()
    ref = rms(x, m.norm.weight) @ m.out.weight.t()
    torch.testing.assert_close(m(ids), ref, rtol=1e-4, atol=1e-4)
