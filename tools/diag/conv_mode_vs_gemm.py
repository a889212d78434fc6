#!/usr/bin/env python3
"""3x3 stride-1 convs of ResNet-50 layers 3 / 4 at the bench batch: gemm.hip's implicit-GEMM conv
mode (conv_gemm / conv_gemm_bn) vs the plain NT GEMM (gemm_nt) on a materialised operand of the
same M x N x K -- what the im2col gather and the BN-statistics epilogue cost. One JSON line per
shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timed(fn, it=10):
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
    B = int(os.environ.get("BATCH", "2560"))
    zero = torch.zeros(256, dtype=torch.bfloat16, device=dev)
    for C, H in ((256, 14), (512, 7), (128, 28)):
        x = torch.randn(B, C, H, H, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(C, 9 * C, device=dev) * (9 * C) ** -0.5).bfloat16().contiguous()
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        M, N, K = B * H * H, C, 9 * C
        t_conv = timed(lambda: L.conv_gemm(x, w, 9, zero))
        t_bn = timed(lambda: L.conv_gemm_bn(x, w, 9, zero, rm, rm, rv, 1e-5, 0.1))
        a = torch.randn(M, K, device=dev).bfloat16()
        ok = bool(L.gemm_nt_ok(M, N, K))
        t_plain = timed(lambda: L.gemm_nt(a, w, 0)) if ok else None
        del a
        fl = 2.0 * M * N * K
        print(json.dumps({"C": C, "H": H, "M": M, "N": N, "K": K,
                          "conv_ms": round(t_conv, 4), "conv_bn_ms": round(t_bn, 4),
                          "plain_gemm_ms": None if t_plain is None else round(t_plain, 4),
                          "conv_pf": round(fl / t_conv / 1e12, 3),
                          "conv_bn_pf": round(fl / t_bn / 1e12, 3),
                          "plain_pf": None if t_plain is None else round(fl / t_plain / 1e12, 3)}),
              flush=True)
        del x, w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
