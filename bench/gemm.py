#!/usr/bin/env python3
"""Own NT GEMM (csrc/kernels/gemm.hip) vs hipBLASLt (torch.matmul / F.linear) on the BERT-base
shapes at the batched 8-worker batch (M = 32 768 tokens) and the per-rank batch (M = 4 096), plus
a square 8192^3 reference. Random operands (uniform [-1, 1)), HIP events, median of reps; the
two implementations are interleaved in one process. One JSON line per shape."""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # (name, M, N, K)
    ("qkv", 32768, 2304, 768), ("oproj", 32768, 768, 768), ("fc1", 32768, 3072, 768),
    ("fc2", 32768, 768, 3072), ("fc1_dgrad", 32768, 768, 3072), ("fc2_dgrad", 32768, 3072, 768),
    ("qkv_r", 4096, 2304, 768), ("fc1_r", 4096, 3072, 768), ("fc2_r", 4096, 768, 3072),
    # the per-rank BERT step (V = 1 x 64 x 128 tokens): outputs 768 wide -> 96 tiles of 256^2
    ("oproj_v1", 8192, 768, 768), ("fc2_v1", 8192, 768, 3072), ("qkv_dgrad_v1", 8192, 768, 2304),
    ("fc1_dgrad_v1", 8192, 768, 3072), ("qkv_v1", 8192, 2304, 768),
    ("sq8k", 8192, 8192, 8192),
]


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    from consensusml_amd.ops.native import lib
    dev = torch.device("cuda", 0)
    rows = []
    for name, M, N, K in SHAPES:
        if a.only and name not in a.only:
            continue
        g = torch.Generator(device=dev).manual_seed(0)
        x = (torch.rand(M, K, generator=g, device=dev) * 2 - 1).bfloat16()
        w = (torch.rand(N, K, generator=g, device=dev) * 2 - 1).bfloat16()
        bias = (torch.rand(N, generator=g, device=dev) * 2 - 1).bfloat16()
        y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        h = torch.empty_like(y)
        flop = 2.0 * M * N * K
        r = {"shape": name, "M": M, "N": N, "K": K}
        L = lib()
        if L.gemm_nt_ok(M, N, K):
            r["own_ms"] = timeit(lambda: L.gemm_nt(x, w, 0, out=y, tile=256), a.reps)
        r["own128_ms"] = timeit(lambda: L.gemm_nt(x, w, 0, out=y, tile=128), a.reps)
        r["pick"] = int(L.gemm_nt_pick(M, N, K))
        r["blas_ms"] = timeit(lambda: torch.matmul(x, w.t(), out=y), a.reps)
        r["own_bias_ms"] = timeit(lambda: L.gemm_nt(x, w, 0, bias=bias, out=y), a.reps)
        r["blas_bias_ms"] = timeit(lambda: F.linear(x, w, bias), a.reps)
        if name.startswith("fc1") and not name.endswith("dgrad"):
            r["own_gelu_ms"] = timeit(lambda: lib().gemm_nt(x, w, 1, bias=bias, aux=h, out=y), a.reps)
            r["blas_gelu_ms"] = timeit(lambda: F.gelu(F.linear(x, w, bias)), a.reps)
        if name == "fc2_dgrad":
            cs = torch.empty(8, N, dtype=torch.bfloat16, device=dev)
            h.copy_(y)
            r["own_dgelu_ms"] = timeit(lambda: lib().gemm_nt(x, w, 2, aux=h, out=y, colsum_out=cs),
                                       a.reps)

            def blas_dgelu():
                g = torch.matmul(x, w.t())
                d = torch.ops.aten.gelu_backward(g, h)
                return lib().colsum_seg(d, 8, cs)
            r["blas_dgelu_ms"] = timeit(blas_dgelu, a.reps)
        for k in list(r):
            if k.endswith("_ms"):
                r[k] = round(r[k], 4)
        if "own_ms" in r:
            r["own_tflops"] = round(flop / r["own_ms"] / 1e9, 1)
        r["own128_tflops"] = round(flop / r["own128_ms"] / 1e9, 1)
        r["blas_tflops"] = round(flop / r["blas_ms"] / 1e9, 1)
        rows.append(r)
        print(json.dumps(r), flush=True)
        del x, w, y, h
        torch.cuda.empty_cache()
    if a.json_out:
        with open(a.json_out, "w") as fh:
            for r in rows:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
