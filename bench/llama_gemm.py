#!/usr/bin/env python3
"""Llama-3-8B linear layers at the 4 x 2048-token step (M = 8192): own kernels vs hipBLASLt for
all three GEMMs of each layer -- forward y = x W^T, data gradient dx = dy W, weight gradient
dW = dy^T x -- on random operands (uniform [-1, 1)), HIP events, median of reps, interleaved in
one process. Own: gemm.hip (NT; the data gradient against the transposed weight, transpose time
reported separately) and wgrad1x1.hip (token rows as NHWC pixels). One JSON line per (shape, op).

  python bench/llama_gemm.py [--only wqkv w2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [("wqkv", 6144, 4096), ("wo", 4096, 4096), ("w13", 28672, 4096), ("w2", 4096, 14336),
          ("out", 128256, 4096)]


def timeit(fn, reps):
    for _ in range(2):
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


def nhwc(t2):
    T, C = t2.shape
    return t2.view(T, 1, 1, C).permute(0, 3, 1, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    from consensusml_amd.ops.native import lib
    L = lib()
    dev = torch.device("cuda", 0)
    M = a.M
    out_rows = []
    for name, N, K in SHAPES:
        if a.only and name not in a.only:
            continue
        g = torch.Generator(device=dev).manual_seed(0)
        x = (torch.rand(M, K, generator=g, device=dev) * 2 - 1).bfloat16()
        w = (torch.rand(N, K, generator=g, device=dev) * 2 - 1).bfloat16()
        dy = (torch.rand(M, N, generator=g, device=dev) * 2 - 1).bfloat16()
        flop = 2.0 * M * N * K
        own_ok = bool(L.gemm_nt_ok(M, N, K))
        rows = []
        r = {"shape": name, "op": "fwd", "M": M, "N": N, "K": K,
             "blas_ms": timeit(lambda: F.linear(x, w), a.reps)}
        if own_ok:
            y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            r["own_ms"] = timeit(lambda: L.gemm_nt(x, w, 0, out=y), a.reps)
            del y
        rows.append(r)
        r = {"shape": name, "op": "dgrad", "M": M, "N": K, "K": N,
             "blas_ms": timeit(lambda: dy @ w, a.reps)}
        if bool(L.gemm_nt_ok(M, K, N)):
            wt = L.transpose_bf16(w)
            r["transpose_ms"] = timeit(lambda: L.transpose_bf16(w), a.reps)
            dx = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
            r["own_ms"] = timeit(lambda: L.gemm_nt(dy, wt, 0, out=dx), a.reps)
            del wt, dx
        rows.append(r)
        r = {"shape": name, "op": "wgrad", "M": N, "N": K, "K": M,
             "blas_ms": timeit(lambda: dy.t() @ x, a.reps)}
        if N % 128 == 0 and K % 128 == 0:
            r["own_ms"] = timeit(lambda: L.wgrad1x1(nhwc(dy), nhwc(x), torch.bfloat16), a.reps)
        # NT forms on transposed operands (dW = (dy^T) (x^T)^T): transposes + gemm.hip / hipBLASLt
        r["transpose_ms"] = timeit(lambda: (L.transpose_bf16(dy), L.transpose_bf16(x)), a.reps)
        dyT, xT = L.transpose_bf16(dy), L.transpose_bf16(x)
        if L.gemm_nt_pick(N, K, M) > 0:
            dw = torch.empty(N, K, dtype=torch.bfloat16, device=dev)
            r["own_nt_ms"] = timeit(lambda: L.gemm_nt(dyT, xT, 0, out=dw), a.reps)
            del dw
        r["blas_nt_ms"] = timeit(lambda: torch.matmul(dyT, xT.t()), a.reps)
        del dyT, xT
        rows.append(r)
        for r in rows:
            for k in list(r):
                if k.endswith("_ms"):
                    r[k] = round(r[k], 4)
            r["blas_tflops"] = round(flop / r["blas_ms"] / 1e9, 1)
            for k in ("own", "own_nt", "blas_nt"):
                if k + "_ms" in r:
                    r[k + "_tflops"] = round(flop / r[k + "_ms"] / 1e9, 1)
            print(json.dumps(r), flush=True)
            out_rows.append(r)
        del x, w, dy
        torch.cuda.empty_cache()
    if a.json_out:
        with open(a.json_out, "w") as fh:
            for r in out_rows:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
