"""Model zoo + synthetic data of each model's shape (no datasets offline).

``build_task(cfg, device, dtype)`` returns the model (cast to the compute dtype, channels_last
for CNNs), a synthetic batch generator and the loss. Families: 2-layer MLP (BASELINE config 1),
ResNet-50, BERT-base (MLM), Llama-3-8B (causal LM), plus tiny variants for tests.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Tuple

import torch
import torch.nn as nn

from ..config import ModelConfig
from ..ops.transformer import cross_entropy
from .mlp import MLP
from .resnet import resnet50, resnet_tiny
from .transformer import bert_base, bert_tiny, llama3_8b, llama_tiny


@dataclass
class Task:
    name: str
    model: nn.Module
    make_batch: Callable[[int, torch.Generator], Tuple[torch.Tensor, torch.Tensor]]
    loss_fn: Callable[[nn.Module, Tuple[torch.Tensor, torch.Tensor]], torch.Tensor]
    samples_per_item: int = 1   # tokens/sample accounting (1 = one image / one row)
    # no cross-sample coupling and every parameter-owning op writes per-worker gradients
    # (ops.worker_grads): virtual workers may run as one batched forward / backward
    batched_workers: bool = False


def _ce(model, batch):
    """Mean cross-entropy; bf16 GPU logits go through the fused HIP kernel (no fp32 copy)."""
    x, y = batch
    return cross_entropy(model(x), y)


def build_task(cfg: ModelConfig, device: torch.device, dtype: torch.dtype = torch.bfloat16,
               seed: int = 0) -> Task:
    torch.manual_seed(seed)
    name = cfg.name
    if name == "mlp":
        model = MLP(cfg.in_features, cfg.hidden, cfg.extra.get("classes", 2))
        classes = cfg.extra.get("classes", 2)
        # fixed teacher so the synthetic task is learnable
        g0 = torch.Generator().manual_seed(1234)
        teacher = torch.randn(cfg.in_features, classes, generator=g0).to(device)

        def make(b, gen):
            x = torch.randn(b, cfg.in_features, generator=gen, device=device)
            y = (x @ teacher).argmax(1)
            return x.to(dtype), y
        return Task(name, model.to(device, dtype), make, _ce)
    if name in ("resnet50", "resnet_tiny"):
        model = resnet50(cfg.num_classes) if name == "resnet50" else resnet_tiny(cfg.num_classes)
        model = model.to(device=device, dtype=dtype, memory_format=torch.channels_last)
        S = cfg.image_size
        if cfg.extra.get("synthetic") == "templates":
            # learnable images (robustness benchmark): one fixed smooth template per class
            # (4x4 noise upsampled to SxS) plus pixel noise of the same scale
            g0 = torch.Generator().manual_seed(4321)
            low = torch.randn(cfg.num_classes, 3, 4, 4, generator=g0)
            tmpl = torch.nn.functional.interpolate(low, size=(S, S), mode="bilinear",
                                                   align_corners=False).to(device)
            noise = float(cfg.extra.get("noise", 1.0))

            def make(b, gen):
                y = torch.randint(0, cfg.num_classes, (b,), generator=gen, device=device)
                x = tmpl[y] + noise * torch.randn(b, 3, S, S, generator=gen, device=device)
                return x.to(dtype).contiguous(memory_format=torch.channels_last), y
            return Task(name, model, make, _ce)

        def make(b, gen):
            x = torch.randn(b, 3, S, S, generator=gen, device=device)
            y = torch.randint(0, cfg.num_classes, (b,), generator=gen, device=device)
            return x.to(dtype).contiguous(memory_format=torch.channels_last), y
        return Task(name, model, make, _ce)
    if name in ("bert_base", "bert_tiny"):
        model = (bert_base() if name == "bert_base" else bert_tiny()).to(device, dtype)
        V = model.c.vocab
        S = cfg.seq_len

        def make(b, gen):
            ids = torch.randint(0, V, (b, S), generator=gen, device=device)
            labels = torch.randint(0, V, (b, S), generator=gen, device=device)
            return ids, labels
        return Task(name, model, make, _ce, samples_per_item=S, batched_workers=True)
    if name in ("llama3_8b", "llama_tiny"):
        model = (llama3_8b() if name == "llama3_8b" else llama_tiny()).to(device, dtype)
        V = model.c.vocab
        S = cfg.seq_len

        def make(b, gen):
            ids = torch.randint(0, V, (b, S + 1), generator=gen, device=device)
            return ids[:, :-1].contiguous(), ids[:, 1:].contiguous()
        return Task(name, model, make, _ce, samples_per_item=S)
    raise ValueError(f"unknown model {name!r}")


__all__ = ["Task", "build_task", "MLP", "resnet50", "resnet_tiny", "bert_base", "bert_tiny",
           "llama3_8b", "llama_tiny"]
