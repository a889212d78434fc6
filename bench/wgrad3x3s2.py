#!/usr/bin/env python3
"""Stride-2 3x3 weight gradients of ResNet-50 (the downsample blocks' conv2) at batch 2048:
wgrad3x3s2.hip vs MIOpen (aten.convolution_backward), median of interleaved reps.

  python bench/wgrad3x3s2.py [--batch 2048] [--reps 10] [--json-out F]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [("l2.0.conv2", 128, 56), ("l3.0.conv2", 256, 28), ("l4.0.conv2", 512, 14)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    from consensusml_amd.ops.native import lib
    L = lib()
    dev = torch.device("cuda")
    g0 = torch.Generator(device=dev).manual_seed(0)
    nh = lambda t: t.contiguous(memory_format=torch.channels_last)   # noqa: E731
    for name, C, H in SHAPES:
        B = a.batch
        x = nh(torch.randn(B, C, H, H, device=dev, generator=g0).bfloat16())
        dy = nh(torch.randn(B, C, H // 2, H // 2, device=dev, generator=g0).bfloat16())
        w = torch.randn(C, C, 3, 3, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        zero = torch.zeros(64, device=dev, dtype=torch.bfloat16)
        fns = [lambda: L.wgrad3x3_s2(dy, x, torch.bfloat16, zero),
               lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [1, 1], [1, 1],
                                                           False, [0, 0], 1, [False, True, False])]
        for f in fns:
            f()
            f()
        torch.cuda.synchronize()
        ts = [[], []]
        for _ in range(a.reps):
            for i, f in enumerate(fns):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                f()
                e1.record()
                e1.synchronize()
                ts[i].append(e0.elapsed_time(e1))
        own, lib_ = (sorted(t)[len(t) // 2] for t in ts)
        fl = 2.0 * B * (H // 2) ** 2 * C * C * 9
        r = {"shape": name, "batch": B, "own_ms": round(own, 4), "miopen_ms": round(lib_, 4),
             "own_tflops": round(fl / own / 1e9, 1), "miopen_tflops": round(fl / lib_ / 1e9, 1)}
        print(json.dumps(r), flush=True)
        if a.json_out:
            with open(a.json_out, "a") as fh:
                fh.write(json.dumps(r) + "\n")
        del x, dy
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
