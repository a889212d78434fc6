#!/usr/bin/env python3
"""Weight gradient of a transformer linear, dW [N, K] = dY^T X over T token rows, on the 1x1-conv
weight-gradient kernel (csrc/kernels/wgrad1x1.hip: the [T, C] row-major activations ARE NHWC
[T, C, 1, 1]; split-K over the rows + fixed-order fold) vs PyTorch's `dy.t() @ x` (hipBLASLt), at
the BERT-base per-rank shapes (T = 64 x 128 or 32 x 128 tokens), or (--llama) the Llama-3-8B
ones at T = 4 x 2048 (wqkv, wo, w13, w2, output head: one split on the LDS-DMA kernel, dW written
directly). Prints one JSON line per shape: times, TFLOP/s and the max relative difference to an
fp32 reference.

  python bench/linear_wgrad.py [--llama]
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _t(fn, it=20):
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


def nhwc(t2: torch.Tensor) -> torch.Tensor:
    """[T, C] contiguous -> the same memory as an NHWC [T, C, 1, 1] tensor."""
    T, C = t2.shape
    return t2.view(T, 1, 1, C).permute(0, 3, 1, 2)


def main():
    from consensusml_amd.ops.native import lib
    L = lib()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    if "--llama" in sys.argv:
        cases = [(8192, (6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096))]
    else:
        cases = [(T, (768, 768), (2304, 768), (3072, 768), (768, 3072)) for T in (8192, 4096)]
    for T, *shapes in cases:
        for N, K in shapes:
            dy = torch.randn(T, N, device=dev, generator=g).bfloat16()
            x = torch.randn(T, K, device=dev, generator=g).bfloat16()
            ref = dy.float().t() @ x.float()
            a = dy.t() @ x
            b = L.wgrad1x1(nhwc(dy), nhwc(x), torch.bfloat16).view(N, K)
            ea = float((a.float() - ref).abs().max() / ref.abs().max())
            eb = float((b.float() - ref).abs().max() / ref.abs().max())
            ta = _t(lambda: dy.t() @ x)
            tb = _t(lambda: L.wgrad1x1(nhwc(dy), nhwc(x), torch.bfloat16))
            # NT on transposed operands (what the bias-free Llama linears do): transposes included
            tc = _t(lambda: torch.matmul(L.transpose_bf16(dy), L.transpose_bf16(x).t()))
            fl = 2.0 * T * N * K
            print(json.dumps({"T": T, "N": N, "K": K, "hipblaslt_us": round(ta * 1e3, 1),
                              "wgrad1x1_us": round(tb * 1e3, 1),
                              "nt_transposed_us": round(tc * 1e3, 1),
                              "hipblaslt_tflops": round(fl / ta / 1e9, 1),
                              "wgrad1x1_tflops": round(fl / tb / 1e9, 1),
                              "nt_transposed_tflops": round(fl / tc / 1e9, 1),
                              "err_hipblaslt": ea, "err_wgrad1x1": eb}), flush=True)


if __name__ == "__main__":
    main()
