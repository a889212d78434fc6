#!/usr/bin/env python3
"""Stem backward at the ResNet-50 bench shape (batch 2048, 224 x 224): the two-pass path
(maxpool_bwd_sum writes the full-resolution pool gradient, stem_wgrad reads it back) vs
stem_wgrad_pool (routed channel sums, then the pool's input gradient gathered from the pooled
gradient inside the weight-gradient kernel).

  python bench/stem_bwd.py [--batch 2048] [--dy2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _t(fn, it=10):
    for _ in range(2):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--dy2", action="store_true")
    a = ap.parse_args()
    from consensusml_amd.ops.native import lib
    from consensusml_amd.ops.stem import pack_stem_weight
    L = lib()
    dev = torch.device("cuda:0")
    N = a.batch
    x = torch.randn(N, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, device=dev) * 0.1).to(torch.bfloat16)
    gam = torch.empty(64, device=dev).uniform_(0.5, 1.5).to(torch.bfloat16)
    bet = torch.empty(64, device=dev).uniform_(-0.2, 0.2).to(torch.bfloat16)
    z, mean, invstd = L.stem_conv_fwd(x, pack_stem_weight(w), None, None, 1e-5, 0.1, True)
    y, idx, _, _ = L.bn_relu_maxpool_fwd(z, gam, bet, None, None, mean, invstd, 1e-5, 0.1,
                                         False, 3, 2, 1)
    dy = torch.randn_like(y)
    dy2 = torch.randn_like(y) if a.dy2 else None

    def two_pass():
        g, gsum = L.maxpool_bwd_sum(dy, idx, z.shape[2], z.shape[3], dy2)
        return L.stem_wgrad(g, z, x, mean, invstd, gam, gsum)

    def gather():
        return L.stem_wgrad_pool(dy, idx, dy2, z, x, mean, invstd, gam)

    r = {"batch": N, "dy2": a.dy2, "two_pass_ms": round(_t(two_pass), 4),
         "gather_ms": round(_t(gather), 4)}
    d1, d2 = two_pass()[0], gather()[0]
    r["dw_rel_diff"] = float((d1 - d2).norm() / d1.norm())
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
