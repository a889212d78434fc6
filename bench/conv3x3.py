#!/usr/bin/env python3
"""3x3 stride-1 convolutions of ResNet-50 at batch 2048: MIOpen (F.conv2d, channels_last bf16)
vs the implicit-GEMM TAP mode of csrc/kernels/conv1x1.hip (with and without the BN + ReLU
prologue and BN statistics epilogue). Prints max error vs an fp32 reference on a slice too.

  python bench/conv3x3.py
"""
from __future__ import annotations

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
    from consensusml_amd.ops.native import lib
    from consensusml_amd.utils.tuning import configure_miopen
    configure_miopen()
    torch.backends.cudnn.benchmark = True
    L = lib()
    dev = torch.device("cuda:0")
    batch = int(os.environ.get("BATCH", "2048"))
    for C, H in ((64, 56), (128, 28), (256, 14), (512, 7)):
        x = torch.randn(batch, C, H, H, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(C, C, 3, 3, device=dev) * (9 * C) ** -0.5).bfloat16().contiguous(
            memory_format=torch.channels_last)
        sc = torch.rand(C, device=dev) + 0.5
        bi = torch.randn(C, device=dev) * 0.1
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        flops = 2 * batch * H * H * 9 * C * C
        t_lib = _t(lambda: F.conv2d(x, w, padding=1))
        t_own = _t(lambda: L.conv3x3_bn_fwd(x, w, None, None, None, None, None, False, 1e-5, 0.1))
        t_own_st = _t(lambda: L.conv3x3_bn_fwd(x, w, sc, bi, rm, rm, rv, True, 1e-5, 0.1))
        # numerics on the first 4 images
        xs = x[:4]
        y, _, _ = L.conv3x3_bn_fwd(xs.contiguous(memory_format=torch.channels_last), w, None, None,
                                   None, None, None, False, 1e-5, 0.1)
        ref = F.conv2d(xs.float(), w.float(), padding=1)
        err = float((y.float() - ref).norm() / ref.norm())
        print(json.dumps({"C": C, "H": H, "batch": batch, "miopen_ms": round(t_lib, 4),
                          "own_ms": round(t_own, 4), "own_bnrelu_stats_ms": round(t_own_st, 4),
                          "miopen_tflops": round(flops / t_lib / 1e9, 1),
                          "own_tflops": round(flops / t_own / 1e9, 1), "rel_err": err}), flush=True)
        del x, w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
