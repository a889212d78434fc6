#!/usr/bin/env python3
"""Optimizer step time: consensusml_amd.optim fused flat-buffer optimizers vs torch.optim
(foreach and, where available, fused=True) on ResNet-50 / BERT-base parameter sets.

  python bench/optim_step.py --model resnet50 --dtype fp32
One JSON line per (optimizer, implementation): ms per step, effective GB/s of state traffic.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _params(model: str, dtype: torch.dtype, dev: torch.device):
    from consensusml_amd.models import bert_base, resnet50
    m = resnet50(1000) if model == "resnet50" else bert_base()
    m = m.to(dev, dtype)
    for p in m.parameters():
        p.grad = torch.randn_like(p) * 1e-3
    return m


def _time(step, iters=20, warm=5):
    for _ in range(warm):
        step()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        step()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "bert_base"])
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    a = ap.parse_args()
    from consensusml_amd.optim import FusedAdamW, FusedSGD
    dev = torch.device("cuda:0")
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16}[a.dtype]
    rows = []
    for name, fused_cls, torch_cls, kw in (
            ("sgd_momentum", FusedSGD, torch.optim.SGD, dict(lr=0.1, momentum=0.9,
                                                             weight_decay=1e-4)),
            ("adamw", FusedAdamW, torch.optim.AdamW, dict(lr=1e-3, weight_decay=0.01))):
        impls = [("consensusml_amd fused flat", lambda ps: fused_cls(ps, **kw)),
                 ("torch foreach", lambda ps: torch_cls(ps, foreach=True, **kw))]
        impls.append(("torch fused", lambda ps: torch_cls(ps, fused=True, **kw)))
        for label, make in impls:
            m = _params(a.model, dt, dev)
            ps = list(m.parameters())
            n = sum(p.numel() for p in ps)
            try:
                opt = make(ps)
                ms = _time(opt.step)
            except (RuntimeError, ValueError, TypeError) as e:
                rows.append({"optimizer": name, "impl": label, "error": str(e)[:120]})
                continue
            # bytes per element: param r/w, grad r, state r/w (+ fp32 master r/w for bf16 fused)
            es = torch.finfo(dt).bits // 8
            nstate = 1 if name.startswith("sgd") else 2
            byts = n * (2 * es + es + nstate * 8)
            if label.startswith("consensusml") and dt != torch.float32:
                byts += n * 8
            rows.append({"optimizer": name, "impl": label, "model": a.model, "dtype": a.dtype,
                         "params": n, "ms_per_step": round(ms, 4),
                         "GBps": round(byts / ms / 1e6, 1)})
            del opt, m, ps
            torch.cuda.empty_cache()
    for r in rows:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
