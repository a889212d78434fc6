#!/usr/bin/env python3
"""ResNet-50's stride-2 convolutions at batch 2048: the downsample 1x1 weight gradient (MIOpen vs
wgrad1x1.hip's stride-2 gather) and the 3x3 stride-2 forward (MIOpen + a BN statistics pass vs
conv_gemm.hip with the statistics in its epilogue). One JSON line per shape.

  python bench/stride2.py [--json-out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

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
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--json-out", default=None)
    args = ap.parse_args()
    from consensusml_amd.ops.native import lib
    from consensusml_amd.utils.tuning import configure_miopen
    configure_miopen()
    torch.backends.cudnn.benchmark = True
    L = lib()
    dev = torch.device("cuda:0")
    B = args.batch
    zero = torch.zeros(64, dtype=torch.bfloat16, device=dev)
    rows = []
    # downsample 1x1 stride-2 weight gradients (cin, cout, input H)
    for ci, co, H in ((256, 512, 56), (512, 1024, 28), (1024, 2048, 14)):
        x = torch.randn(B, ci, H, H, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        gy = torch.randn(B, co, H // 2, H // 2, device=dev).bfloat16().contiguous(
            memory_format=torch.channels_last)
        w = torch.zeros(co, ci, 1, 1, device=dev, dtype=torch.bfloat16)
        t_lib = _t(lambda: torch.ops.aten.convolution_backward(
            gy, x, w, None, [2, 2], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False]))
        t_own = _t(lambda: L.wgrad1x1_s2(gy, x, torch.bfloat16))
        r = {"op": "wgrad1x1_s2", "cin": ci, "cout": co, "H": H, "miopen_ms": round(t_lib, 4),
             "own_ms": round(t_own, 4)}
        print(json.dumps(r), flush=True)
        rows.append(r)
        del x, gy
        torch.cuda.empty_cache()
    # 3x3 stride-2 forward (+ BN statistics)
    for C, H in ((128, 56), (256, 28), (512, 14)):
        x = torch.randn(B, C, H, H, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(C, C, 3, 3, device=dev) * (9 * C) ** -0.5).bfloat16().contiguous(
            memory_format=torch.channels_last)
        wf = w.permute(0, 2, 3, 1).reshape(C, 9 * C).contiguous()
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        y = F.conv2d(x, w, padding=1, stride=2)
        t_lib = _t(lambda: F.conv2d(x, w, padding=1, stride=2))
        t_st = _t(lambda: L.bn_stats(y, rm, rv, 1e-5, 0.1))
        t_own = _t(lambda: L.conv_gemm_bn(x, wf, 9, zero, rm, rm, rv, 1e-5, 0.1, 2))
        t_own_plain = _t(lambda: L.conv_gemm(x, wf, 9, zero, 2))
        flops = 2 * B * (H // 2) ** 2 * 9 * C * C
        r = {"op": "conv3x3_s2_fwd", "C": C, "H": H, "miopen_ms": round(t_lib, 4),
             "bn_stats_ms": round(t_st, 4), "own_bn_ms": round(t_own, 4),
             "own_ms": round(t_own_plain, 4),
             "miopen_pflops": round(flops / t_lib / 1e12, 3),
             "own_pflops": round(flops / t_own_plain / 1e12, 3)}
        print(json.dumps(r), flush=True)
        rows.append(r)
        del x, y
        torch.cuda.empty_cache()
    if args.json_out:
        with open(args.json_out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
