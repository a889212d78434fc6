"""BERT-base and Llama-3 transformer families (N12).

Attention goes through ``F.scaled_dot_product_attention`` (the ROCm flash / memory-efficient
kernels of PyTorch) — the north star keeps model compute in PyTorch and puts the hand-written
HIP work into aggregation and the optimizer. Random-init weights (no checkpoints offline).

BERT-base: 12 layers, d 768, 12 heads, FFN 3072, vocab 30522, post-LN, GELU, MLM head tied to
the token embedding. Llama-3-8B: 32 layers, d 4096, 32 q / 8 kv heads (GQA), SwiGLU FFN 14336,
RMSNorm, RoPE theta 500000, vocab 128256, untied output head.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F


# =============================================================================== BERT
@dataclass
class BertConfig:
    vocab: int = 30522
    d: int = 768
    layers: int = 12
    heads: int = 12
    ffn: int = 3072
    max_pos: int = 512
    dropout: float = 0.0


class BertLayer(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.h = c.heads
        self.qkv = nn.Linear(c.d, 3 * c.d)
        self.o = nn.Linear(c.d, c.d)
        self.ln1 = nn.LayerNorm(c.d, eps=1e-12)
        self.fc1 = nn.Linear(c.d, c.ffn)
        self.fc2 = nn.Linear(c.ffn, c.d)
        self.ln2 = nn.LayerNorm(c.d, eps=1e-12)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, S, D = x.shape
        q, k, v = self.qkv(x).view(B, S, 3, self.h, D // self.h).permute(2, 0, 3, 1, 4)
        a = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, S, D)
        x = self.ln1(x + self.o(a))
        return self.ln2(x + self.fc2(F.gelu(self.fc1(x))))


class BertMLM(nn.Module):
    def __init__(self, c: BertConfig = BertConfig()):
        super().__init__()
        self.c = c
        self.tok = nn.Embedding(c.vocab, c.d)
        self.pos = nn.Embedding(c.max_pos, c.d)
        self.typ = nn.Embedding(2, c.d)
        self.ln = nn.LayerNorm(c.d, eps=1e-12)
        self.layers = nn.ModuleList([BertLayer(c) for _ in range(c.layers)])
        self.head = nn.Linear(c.d, c.d)
        self.head_ln = nn.LayerNorm(c.d, eps=1e-12)
        self.bias = nn.Parameter(torch.zeros(c.vocab))
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, std=0.02)
                if isinstance(m, nn.Linear) and m.bias is not None:
                    nn.init.zeros_(m.bias)

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        B, S = ids.shape
        pos = torch.arange(S, device=ids.device)
        x = self.tok(ids) + self.pos(pos)[None] + self.typ.weight[0]
        x = self.ln(x)
        for l in self.layers:
            x = l(x)
        x = self.head_ln(F.gelu(self.head(x)))
        return F.linear(x, self.tok.weight, self.bias)


def bert_base() -> BertMLM:
    return BertMLM(BertConfig())


def bert_tiny() -> BertMLM:
    return BertMLM(BertConfig(vocab=512, d=64, layers=2, heads=4, ffn=128, max_pos=128))


# =============================================================================== Llama
@dataclass
class LlamaConfig:
    vocab: int = 128256
    d: int = 4096
    layers: int = 32
    heads: int = 32
    kv_heads: int = 8
    ffn: int = 14336
    rope_theta: float = 500000.0
    eps: float = 1e-5
    max_seq: int = 8192


class RMSNorm(nn.Module):
    def __init__(self, d: int, eps: float):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(d))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        xf = x.float()
        xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps)
        return xf.to(x.dtype) * self.weight


def rope_cache(S: int, hd: int, theta: float, device, dtype):
    inv = 1.0 / (theta ** (torch.arange(0, hd, 2, device=device, dtype=torch.float32) / hd))
    t = torch.arange(S, device=device, dtype=torch.float32)
    f = torch.outer(t, inv)
    return f.cos().to(dtype), f.sin().to(dtype)


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    x1, x2 = x[..., 0::2], x[..., 1::2]
    c, s = cos[None, None], sin[None, None]
    out = torch.stack((x1 * c - x2 * s, x1 * s + x2 * c), -1)
    return out.flatten(-2)


class LlamaBlock(nn.Module):
    def __init__(self, c: LlamaConfig):
        super().__init__()
        self.c = c
        hd = c.d // c.heads
        self.hd = hd
        self.wq = nn.Linear(c.d, c.heads * hd, bias=False)
        self.wk = nn.Linear(c.d, c.kv_heads * hd, bias=False)
        self.wv = nn.Linear(c.d, c.kv_heads * hd, bias=False)
        self.wo = nn.Linear(c.heads * hd, c.d, bias=False)
        self.w1 = nn.Linear(c.d, c.ffn, bias=False)
        self.w3 = nn.Linear(c.d, c.ffn, bias=False)
        self.w2 = nn.Linear(c.ffn, c.d, bias=False)
        self.n1 = RMSNorm(c.d, c.eps)
        self.n2 = RMSNorm(c.d, c.eps)

    def forward(self, x, cos, sin):
        B, S, D = x.shape
        h = self.n1(x)
        q = self.wq(h).view(B, S, self.c.heads, self.hd).transpose(1, 2)
        k = self.wk(h).view(B, S, self.c.kv_heads, self.hd).transpose(1, 2)
        v = self.wv(h).view(B, S, self.c.kv_heads, self.hd).transpose(1, 2)
        q, k = apply_rope(q, cos, sin), apply_rope(k, cos, sin)
        a = F.scaled_dot_product_attention(q, k, v, is_causal=True,
                                           enable_gqa=self.c.heads != self.c.kv_heads)
        x = x + self.wo(a.transpose(1, 2).reshape(B, S, D))
        h = self.n2(x)
        return x + self.w2(F.silu(self.w1(h)) * self.w3(h))


class Llama(nn.Module):
    def __init__(self, c: LlamaConfig = LlamaConfig(), checkpoint_layers: bool = False):
        super().__init__()
        self.c = c
        self.ckpt = checkpoint_layers
        self.tok = nn.Embedding(c.vocab, c.d)
        self.layers = nn.ModuleList([LlamaBlock(c) for _ in range(c.layers)])
        self.norm = RMSNorm(c.d, c.eps)
        self.out = nn.Linear(c.d, c.vocab, bias=False)
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, std=0.02)

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        B, S = ids.shape
        x = self.tok(ids)
        cos, sin = rope_cache(S, self.c.d // self.c.heads, self.c.rope_theta, ids.device, x.dtype)
        for l in self.layers:
            if self.ckpt and self.training:
                x = torch.utils.checkpoint.checkpoint(l, x, cos, sin, use_reentrant=False)
            else:
                x = l(x, cos, sin)
        return self.out(self.norm(x))


def llama3_8b(checkpoint_layers: bool = True) -> Llama:
    return Llama(LlamaConfig(), checkpoint_layers)


def llama_tiny() -> Llama:
    return Llama(LlamaConfig(vocab=512, d=64, layers=2, heads=4, kv_heads=2, ffn=128, max_seq=256))
