#!/usr/bin/env python3
"""1x1-conv data-gradient GEMMs of ResNet-50 at batch 2048: hipBLASLt (torch.mm / addmm, the
model's current path on layers 3-4) vs conv_gemm.hip with taps = 1.

  python bench/gemm1x1.py
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
    B = 2048
    # (name, H, K (input channels of the GEMM), N (output channels))
    shapes = [("l2_conv1_dgrad", 28, 128, 512), ("l2_conv3_dgrad", 28, 512, 128),
              ("l3_conv1_dgrad", 14, 256, 1024), ("l3_conv3_dgrad", 14, 1024, 256),
              ("l4_conv1_dgrad", 7, 512, 2048), ("l4_conv3_dgrad", 7, 2048, 512)]
    for name, H, K, N in shapes:
        M = B * H * H
        x = torch.randn(B, K, H, H, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(N, K, device=dev) * K ** -0.5).bfloat16()
        x2 = x.permute(0, 2, 3, 1).reshape(M, K)
        t_mm = _t(lambda: torch.mm(x2, w.t()))
        t_g = _t(lambda: L.conv_gemm(x, w, 1))
        y = L.conv_gemm(x, w, 1)
        ref = torch.mm(x2.float()[:4096], w.float().t())
        err = float((y.permute(0, 2, 3, 1).reshape(M, N)[:4096].float() - ref).norm() / ref.norm())
        fl = 2 * M * K * N
        print(json.dumps({"shape": name, "M": M, "K": K, "N": N, "hipblaslt_ms": round(t_mm, 4),
                          "conv_gemm_ms": round(t_g, 4), "hipblaslt_tflops": round(fl / t_mm / 1e9, 1),
                          "conv_gemm_tflops": round(fl / t_g / 1e9, 1), "rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
