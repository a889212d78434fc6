#!/usr/bin/env python3
"""ResNet-50 stem (7x7 stride-2 conv, 3 -> 64 channels, batch B at 224x224, bf16 NHWC) forward +
weight gradient on MIOpen with the input channels zero-padded to 3 / 4 / 8: Cin = 3 rules out
MIOpen's vectorised NHWC kernels. One JSON line per padding with ms per pass."""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    a = ap.parse_args()
    from consensusml_amd.utils.tuning import configure_miopen
    configure_miopen()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    B = a.batch
    for cin in (3, 4, 8):
        x = torch.randn(B, cin, 224, 224, device=dev, dtype=torch.bfloat16)
        x = x.contiguous(memory_format=torch.channels_last)
        w = torch.randn(64, cin, 7, 7, device=dev, dtype=torch.bfloat16)
        w = w.contiguous(memory_format=torch.channels_last)
        y = F.conv2d(x, w, stride=2, padding=3)
        dy = torch.randn_like(y)
        fwd = timeit(lambda: F.conv2d(x, w, stride=2, padding=3))
        wg = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1, [False, True, False]))
        pad = timeit(lambda: F.pad(x[:, :3], (0, 0, 0, 0, 0, cin - 3)) if cin > 3 else x)
        print(json.dumps({"cin": cin, "batch": B, "fwd_ms": round(fwd, 4), "wgrad_ms": round(wg, 4),
                          "pad_ms": round(pad, 4)}), flush=True)


if __name__ == "__main__":
    main()
