#!/usr/bin/env python3
"""Backward 1x1 data-gradient kernels of the fused identity-block tails at the ResNet-50 batch-2048
shapes (csrc/kernels/conv1x1.hip): ``conv1x1_link`` (dX = dY W^T + masked residual gradient,
optionally + the producer BN's backward sums) and ``conv1x1_bnbwd`` (BN-backward prologue), vs the
plain hipBLASLt GEMM of the same product. Prints ms and effective HBM bandwidth (minimum bytes:
every operand read once, the output written once).

  python bench/link_kernels.py
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


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def main():
    from consensusml_amd.ops.native import lib
    L = lib()
    dev = torch.device("cuda:0")
    batch = int(os.environ.get("BATCH", "2048"))
    for planes, H in ((64, 56), (128, 28), (256, 14), (512, 7)):
        K, N = planes, 4 * planes           # conv1 dgrad: dy1 [M, planes] -> dx [M, 4 planes]
        M = batch * H * H
        dy = _nhwc(torch.randn(batch, K, H, H, device=dev).bfloat16())
        wt = (torch.randn(N, K, device=dev) * K ** -0.5).bfloat16()    # [N][K]: y = dy wt^T
        link = _nhwc(torch.randn(batch, N, H, H, device=dev).bfloat16())
        lm = torch.randint(0, 256, (M, N // 8), device=dev, dtype=torch.uint8)
        sz = _nhwc(torch.randn(batch, N, H, H, device=dev).bfloat16())
        sm = torch.randint(0, 256, (M, N // 8), device=dev, dtype=torch.uint8)
        mean = torch.zeros(N, device=dev)
        invstd = torch.ones(N, device=dev)
        b2, b1 = 2, 1
        t_link = _t(lambda: L.conv1x1_link(dy, wt, link, lm))
        t_sums = _t(lambda: L.conv1x1_link(dy, wt, link, lm, sz, sm, mean, invstd))
        dy2 = dy.permute(0, 2, 3, 1).reshape(M, K)
        wk = wt.t().contiguous()
        t_mm = _t(lambda: torch.mm(dy2, wk))
        by_link = M * K * b2 + M * N * (b2 + b2) + M * N // 8 * b1
        by_sums = by_link + M * N * b2 + M * N // 8 * b1
        by_mm = M * K * b2 + M * N * b2
        # conv3 dgrad of the fused tail: dz3 = a (m ? g : 0) + b z3 + c on load, [M, 4p] -> [M, p]
        g = link
        ca, cb, cc = (torch.randn(N, device=dev) for _ in range(3))
        w3 = (torch.randn(K, N, device=dev) * N ** -0.5).bfloat16()      # [p][4p]: [out][red]
        t_bnbwd = _t(lambda: L.conv1x1_bnbwd(g, sz, sm, ca, cb, cc, w3))
        by_bnbwd = M * N * (b2 + b2) + M * N // 8 * b1 + M * K * b2
        w3t = w3.t().contiguous()
        t_mm3 = _t(lambda: torch.mm(g.permute(0, 2, 3, 1).reshape(M, N), w3t))
        del wk
        r = {"planes": planes, "H": H, "batch": batch,
             "link_ms": round(t_link, 4), "link_TBps": round(by_link / t_link / 1e9, 2),
             "link_sums_ms": round(t_sums, 4), "link_sums_TBps": round(by_sums / t_sums / 1e9, 2),
             "gemm_ms": round(t_mm, 4), "gemm_TBps": round(by_mm / t_mm / 1e9, 2),
             "bnbwd_ms": round(t_bnbwd, 4), "bnbwd_TBps": round(by_bnbwd / t_bnbwd / 1e9, 2),
             "gemm3_ms": round(t_mm3, 4)}
        print(json.dumps(r), flush=True)
        del dy, link, lm, sz, sm, g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
