#!/usr/bin/env python3
"""gemm_w4.hip (4 waves x 128 x 128 per 256 x 256 tile, any operand layout) vs hipBLASLt and the
8-wave gemm.hip on the square 8192^3 / 4096^3 shapes and the Llama-3-8B linear layers at the
4 x 2048-token step (M = 8192): forward y = x W^T (mode 0), data gradient dx = dy W (mode 2, W read
k-major in place), weight gradient dW = dy^T x (mode 3, both operands k-major in place). Random
operands (uniform [-1, 1)), HIP events, median of reps; own and library arms interleaved in one
process (cdna_hip_programming.md rule 24). One JSON line per (shape, op), with the max abs error
of the own result against hipBLASLt's.

  python bench/gemm_w4.py [--only sq8k wqkv] [--ops fwd wgrad]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

LLAMA = [("wqkv", 6144, 4096), ("wo", 4096, 4096), ("w13", 28672, 4096), ("w2", 4096, 14336),
         ("out", 128256, 4096)]


def timeit(fns, reps):
    """fns: dict name -> callable; interleaved rounds, median ms per name."""
    for f in fns.values():
        f()
        f()
    torch.cuda.synchronize()
    ts = {k: [] for k in fns}
    for _ in range(reps):
        for k, f in fns.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            f()
            b.record()
            torch.cuda.synchronize()
            ts[k].append(a.elapsed_time(b))
    return {k: sorted(v)[len(v) // 2] for k, v in ts.items()}


def rnd(shape, g, dev):
    return (torch.rand(*shape, generator=g, device=dev) * 2 - 1).bfloat16()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--ops", nargs="*", default=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    from consensusml_amd.ops.native import lib
    L = lib()
    dev = torch.device("cuda", 0)
    rows = []

    def emit(r, flop):
        for k in list(r):
            if k.endswith("_ms"):
                r[k] = round(r[k], 4)
                r[k[:-3] + "_tflops"] = round(flop / r[k] / 1e9, 1)
        print(json.dumps(r), flush=True)
        rows.append(r)

    for name, n in (("sq8k", 8192), ("sq4k", 4096)):
        if a.only and name not in a.only:
            continue
        g = torch.Generator(device=dev).manual_seed(0)
        x, w = rnd((n, n), g, dev), rnd((n, n), g, dev)
        y = torch.empty(n, n, dtype=torch.bfloat16, device=dev)
        y2 = torch.empty_like(y)
        t = timeit({"w4": lambda: L.gemm_w4(x, w, 0, out=y), "blas": lambda: torch.matmul(x, w.t(), out=y2),
                    "gemm8w": lambda: L.gemm_nt(x, w, 0, out=y2, tile=256)}, a.reps)
        L.gemm_w4(x, w, 0, out=y)
        torch.matmul(x, w.t(), out=y2)
        r = {"shape": name, "op": "fwd", "M": n, "N": n, "K": n, **{k + "_ms": v for k, v in t.items()},
             "max_err_vs_blas": float((y.float() - y2.float()).abs().max())}
        emit(r, 2.0 * n ** 3)
        del x, w, y, y2
    M = a.M
    for name, N, K in LLAMA:
        if a.only and name not in a.only:
            continue
        g = torch.Generator(device=dev).manual_seed(0)
        x, w, dy = rnd((M, K), g, dev), rnd((N, K), g, dev), rnd((M, N), g, dev)
        flop = 2.0 * M * N * K
        if "fwd" in a.ops:
            y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            t = timeit({"w4": lambda: L.gemm_w4(x, w, 0, out=y), "blas": lambda: F.linear(x, w)}, a.reps)
            ref = F.linear(x, w)
            L.gemm_w4(x, w, 0, out=y)
            emit({"shape": name, "op": "fwd", "M": M, "N": N, "K": K, **{k + "_ms": v for k, v in t.items()},
                  "max_err_vs_blas": float((y.float() - ref.float()).abs().max())}, flop)
            del y, ref
        if "dgrad" in a.ops:
            dx = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
            t = timeit({"w4": lambda: L.gemm_w4(dy, w, 2, out=dx), "blas": lambda: dy @ w}, a.reps)
            ref = dy @ w
            L.gemm_w4(dy, w, 2, out=dx)
            emit({"shape": name, "op": "dgrad", "M": M, "N": K, "K": N, **{k + "_ms": v for k, v in t.items()},
                  "max_err_vs_blas": float((dx.float() - ref.float()).abs().max())}, flop)
            del dx, ref
        if "wgrad" in a.ops:
            dw = torch.empty(N, K, dtype=torch.bfloat16, device=dev)

            def blas_nt():   # the round-5 path: two transposes + hipBLASLt NT
                return torch.matmul(L.transpose_bf16(dy), L.transpose_bf16(x).t())
            t = timeit({"w4": lambda: L.gemm_w4(dy, x, 3, out=dw), "blas": lambda: dy.t() @ x,
                        "blas_nt": blas_nt}, a.reps)
            ref = dy.t() @ x
            L.gemm_w4(dy, x, 3, out=dw)
            emit({"shape": name, "op": "wgrad", "M": N, "N": K, "K": M, **{k + "_ms": v for k, v in t.items()},
                  "max_err_vs_blas": float((dw.float() - ref.float()).abs().max())}, flop)
            del dw, ref
        del x, w, dy
        torch.cuda.empty_cache()
    if a.json_out:
        with open(a.json_out, "w") as fh:
            for r in rows:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
