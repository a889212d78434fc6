"""BERT-base and Llama-3 transformer families (N12).

Attention runs own MFMA kernels: BERT's short sequences ``csrc/kernels/attention.hip``, Llama's
causal GQA attention (head dim 128) ``csrc/kernels/flash_attn.hip`` forward and backward. The
GEMMs are gemm.hip or hipBLASLt. Everything between them runs the hand-written HIP kernels of
``csrc/kernels/transformer.hip`` (``ops.transformer``) on bf16 GPU tensors:
  * the q / k / v projections are ONE fused GEMM. BERT's attention (S <= 128, head dim 64) runs
    the MFMA kernel of ``csrc/kernels/attention.hip`` straight from that fused output to the
    output projection's input layout; Llama's is split and rotated into head-major q / k / v by
    one kernel, the flash kernels write O in the output projection's row layout, and the backward
    returns through one RoPE-backward kernel that also sums the GQA group's dk / dv;
  * every residual add is fused with the following norm (``add_norm``: the residual stream and the
    normalised sublayer input come out of one pass, and the backward adds the stream's gradient
    on the way out);
  * Llama's gate / up projections are one GEMM feeding a one-pass SwiGLU;
  * linear-layer bias gradients use a bandwidth-bound column-sum kernel;
  * the loss is the fused bf16 cross-entropy (``models.build_task``).
CPU / fp32 tensors run the PyTorch compositions of the same ops.

BERT-base: 12 layers, d 768, 12 heads, FFN 3072, vocab 30522, post-LN, GELU, MLM head tied to
the token embedding. Llama-3-8B: 32 layers, d 4096, 32 q / 8 kv heads (GQA), SwiGLU FFN 14336,
RMSNorm, RoPE theta 500000 (interleaved pairs), vocab 128256, untied output head.
Random-init weights (no checkpoints offline).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn as nn

from ..ops.bn import ResidualLink
from ..ops.transformer import (LayerNorm, Linear, LinearNB, RMSNorm, add_norm, bert_embed,
                               ffn_gelu, fused_qkv_attention, linear, linear_gelu, qkv_attention,
                               rope_tables, swiglu)


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
        self.qkv = Linear(c.d, 3 * c.d)
        self.o = Linear(c.d, c.d)
        self.ln1 = LayerNorm(c.d, eps=1e-12)
        self.fc1 = Linear(c.d, c.ffn)
        self.fc2 = Linear(c.ffn, c.d)
        self.ln2 = LayerNorm(c.d, eps=1e-12)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, S, D = x.shape
        # x feeds both the QKV GEMM and the residual add of ln1 (likewise fc1 / ln2): the norm's
        # backward parks x's residual gradient on a link and the GEMM's data gradient absorbs it
        l1, l2 = ResidualLink(), ResidualLink()
        a = fused_qkv_attention(self.qkv(x, l1), self.h, D // self.h)
        _, x = add_norm(x, self.o(a), self.ln1.weight, self.ln1.bias, self.ln1.eps, l1)  # post-LN
        _, x = add_norm(x, ffn_gelu(x, self.fc1, self.fc2, l2), self.ln2.weight, self.ln2.bias,
                        self.ln2.eps, l2)
        return x


class BertMLM(nn.Module):
    def __init__(self, c: BertConfig = BertConfig()):
        super().__init__()
        self.c = c
        self.tok = nn.Embedding(c.vocab, c.d)
        self.pos = nn.Embedding(c.max_pos, c.d)
        self.typ = nn.Embedding(2, c.d)
        self.ln = LayerNorm(c.d, eps=1e-12)
        self.layers = nn.ModuleList([BertLayer(c) for _ in range(c.layers)])
        self.head = Linear(c.d, c.d)
        self.head_ln = LayerNorm(c.d, eps=1e-12)
        self.bias = nn.Parameter(torch.zeros(c.vocab))
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, std=0.02)
                if isinstance(m, nn.Linear) and m.bias is not None:
                    nn.init.zeros_(m.bias)

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        x = self.ln(bert_embed(ids, self.tok.weight, self.pos.weight, self.typ.weight))
        for l in self.layers:
            x = l(x)
        x = self.head_ln(linear_gelu(x, self.head))
        return linear(x, self.tok.weight, self.bias, logits=True)


def bert_base() -> BertMLM:
    return BertMLM(BertConfig())


def bert_tiny() -> BertMLM:
    # vocab not a multiple of 8 (like BERT-base's 30522): tests cover the padded-logits head
    return BertMLM(BertConfig(vocab=510, d=64, layers=2, heads=4, ffn=128, max_pos=128))


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


class LlamaBlock(nn.Module):
    """Pre-norm block. The residual add that ends a block is fused with the next norm, so a block
    takes (x, m): the residual stream before the previous block's MLP output m was added
    (m = None for the first block), and returns its own (x, m)."""

    def __init__(self, c: LlamaConfig):
        super().__init__()
        self.c = c
        hd = c.d // c.heads
        self.hd = hd
        self.wqkv = LinearNB(c.d, (c.heads + 2 * c.kv_heads) * hd)
        self.wo = LinearNB(c.heads * hd, c.d)
        self.w13 = LinearNB(c.d, 2 * c.ffn)   # [gate | up]
        self.w2 = LinearNB(c.ffn, c.d)
        self.n1 = RMSNorm(c.d, c.eps)
        self.n2 = RMSNorm(c.d, c.eps)

    def forward(self, x, m, cos, sin):
        B, S, D = x.shape
        x, h = add_norm(x, m, self.n1.weight, None, self.c.eps)
        a = qkv_attention(self.wqkv(h), self.c.heads, self.c.kv_heads, self.hd, cos, sin)
        x, h = add_norm(x, self.wo(a), self.n2.weight, None, self.c.eps)
        return x, self.w2(swiglu(self.w13(h)))


class Llama(nn.Module):
    def __init__(self, c: LlamaConfig = LlamaConfig(), checkpoint_layers: bool = False):
        super().__init__()
        self.c = c
        self.ckpt = checkpoint_layers
        self.tok = nn.Embedding(c.vocab, c.d)
        self.layers = nn.ModuleList([LlamaBlock(c) for _ in range(c.layers)])
        self.norm = RMSNorm(c.d, c.eps)
        self.out = LinearNB(c.d, c.vocab)
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, std=0.02)

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        B, S = ids.shape
        x = self.tok(ids)
        cos, sin = rope_tables(S, self.c.d // self.c.heads, self.c.rope_theta, ids.device)
        m = None
        for l in self.layers:
            if self.ckpt and self.training:
                x, m = torch.utils.checkpoint.checkpoint(l, x, m, cos, sin, use_reentrant=False)
            else:
                x, m = l(x, m, cos, sin)
        _, h = add_norm(x, m, self.norm.weight, None, self.c.eps)
        return self.out(h)


def llama3_8b(checkpoint_layers: bool = False) -> Llama:
    """Without activation checkpointing by default: at 2048 tokens per replica the saved
    activations are ~11 GB, and bf16 params + fp32 master + AdamW state + flat grads + gossip
    buffers come to ~160 GB, well inside 288 GB of HBM3E — recomputing the forward would cost a
    third more GEMM work for memory the MI355X does not need back."""
    return Llama(LlamaConfig(), checkpoint_layers)


def llama_tiny() -> Llama:
    return Llama(LlamaConfig(vocab=512, d=64, layers=2, heads=4, kv_heads=2, ffn=128, max_seq=256))
