#!/usr/bin/env python3
"""Bandwidth of the fused BatchNorm kernels (csrc/kernels/bn_act.hip) at the ResNet-50 batch-2048
activation shapes: bytes moved per call / time -> TB/s (achievable HBM3E ~6.3 TB/s).

  python bench/bn_kernels.py

Measured (profiles/r02_bn_kernels17.jsonl): reductions 5.6-5.9 TB/s, apply passes 4.6-5.3 TB/s.
Apply-pass variants with 4 rows in flight per thread and/or non-temporal stores were within
+-0.2 TB/s of the 2-row version at every shape (profiles/r02_bn_apply_variants18.jsonl) and were
dropped.
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _t(fn, it=10):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    from consensusml_amd.ops.native import lib
    L = lib()
    dev = torch.device("cuda:0")
    shapes = [(2048, 256, 56), (2048, 64, 56), (2048, 512, 28), (2048, 128, 28), (2048, 1024, 14)]
    for N, C, H in shapes:
        M = N * H * H
        nb = M * C * 2
        x = torch.randn(N, C, H, H, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        r = torch.randn_like(x)
        g = torch.randn_like(x)
        gm = torch.ones(C, device=dev).bfloat16()
        bt = torch.zeros(C, device=dev).bfloat16()
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        y, mean, invstd, mask = L.bn_fwd(x, r, gm, bt, rm, rv, None, None, 1e-5, 0.1, True, True, True)
        rows = []
        ms = _t(lambda: L.bn_fwd(x, r, gm, bt, None, None, mean, invstd, 1e-5, 0.1, True, False, True))
        rows.append(("apply res+relu+mask", ms, 3 * nb + nb / 16))
        ms = _t(lambda: L.bn_fwd(x, None, gm, bt, None, None, mean, invstd, 1e-5, 0.1, True, False, False))
        rows.append(("apply relu", ms, 2 * nb))
        ms = _t(lambda: L.bn_stats(x, None, None, 1e-5, 0.1))
        rows.append(("stats", ms, nb))
        ms = _t(lambda: L.bn_bwd(g, None, x, mask, gm, bt, mean, invstd, True, True))
        rows.append(("bwd mask+dres (reduce+apply)", ms, (2 * nb + nb / 16) + (2 * nb + nb / 16 + 2 * nb)))
        ms = _t(lambda: L.bn_bwd_sums(g, None, x, mask, gm, bt, mean, invstd, True))
        rows.append(("bwd reduce mask", ms, 2 * nb + nb / 16))
        ms = _t(lambda: L.bn_bwd(g, None, x, None, gm, bt, mean, invstd, True, False))
        rows.append(("bwd relu-recompute (reduce+apply)", ms, 2 * nb + 3 * nb))
        for name, ms, b in rows:
            print(json.dumps({"shape": f"{N}x{C}x{H}x{H}", "kernel": name, "ms": round(ms, 4),
                              "TBps": round(b / ms / 1e9, 2)}), flush=True)
        del x, r, g, y, mask
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
