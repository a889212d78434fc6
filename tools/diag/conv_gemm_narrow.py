#!/usr/bin/env python3
"""Time conv_gemm.hip on the ResNet-50 layer-1 3x3 shape (64 -> 64 channels, 56 x 56, batch 2048)
under the CML_CONV_GEMM_NARROW variant of this process; one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from consensusml_amd.ops.native import lib
    L = lib()
    dev = torch.device("cuda:0")
    B, C, H = int(os.environ.get("BATCH", "2048")), 64, 56
    x = torch.randn(B, C, H, H, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(C, 9 * C, device=dev) * (9 * C) ** -0.5).bfloat16().contiguous()
    zero = torch.zeros(64, dtype=torch.bfloat16, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    for _ in range(3):
        L.conv_gemm(x, w, 9, zero)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(10):
        L.conv_gemm(x, w, 9, zero)
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) / 10
    s.record()
    for _ in range(10):
        L.conv_gemm_bn(x, w, 9, zero, rm, rm, rv, 1e-5, 0.1)
    e.record()
    torch.cuda.synchronize()
    tb = s.elapsed_time(e) / 10
    xs = x[:2].contiguous(memory_format=torch.channels_last)
    y = L.conv_gemm(xs, w, 9, zero)
    ref = torch.nn.functional.conv2d(xs.float(), w.view(C, 3, 3, C).permute(0, 3, 1, 2).float(),
                                     padding=1)
    err = float((y.float() - ref).norm() / ref.norm())
    flops = 2 * B * H * H * 9 * C * C
    print(json.dumps({"variant": os.environ.get("CML_CONV_GEMM_NARROW", "0"), "ms": round(t, 4),
                      "bn_ms": round(tb, 4), "pflops": round(flops / t / 1e12, 3),
                      "rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
