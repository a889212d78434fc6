#!/usr/bin/env python3
"""Micro-benchmark of the aggregation hot path at ResNet-50 / BERT sizes on one MI355X.

For n workers x D coordinates (bf16), times (HIP events, median of reps):
  gram           G = X X^T (MFMA split-K + fp64 reduce)
  weights        Krum / Weiszfeld weights on G (one wave)
  median_sgd     coordinate median fused with SGD-momentum (master, momentum, bf16 params)
  trimmed_sgd    trimmed mean (trim f) fused with SGD-momentum
  krum_sgd       weighted combine (one-hot Krum weights: 1 row read) fused with SGD-momentum
  mean_sgd       weighted combine of all n rows fused with SGD-momentum
and the PyTorch equivalents (torch.median / sort / matmul / foreach) for comparison. Reports
achieved HBM GB/s from the bytes each kernel must move. One JSON line per (n, D).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps: int = 20) -> float:
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
    ap.add_argument("--n", type=int, nargs="*", default=[4, 8, 16])
    # ResNet-50 / BERT-base parameter counts, rounded up to the engine's 64-element bucket padding
    # (a row stride that is not a multiple of 8 bf16 would make gram() copy X to a padded buffer)
    ap.add_argument("--D", type=int, nargs="*", default=[25_557_032, 109_514_304])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    from consensusml_amd.ops import kernels as K
    dev = torch.device("cuda", 0)
    for D in a.D:
        for n in a.n:
            g = torch.Generator(device=dev).manual_seed(0)
            X = torch.randn(n, D, generator=g, device=dev).to(torch.bfloat16)
            master = torch.randn(D, device=dev)
            mom = torch.zeros(D, device=dev)
            p = torch.empty(D, dtype=torch.bfloat16, device=dev)
            opt = K.OptArgs(kind="sgd", lr=0.1, momentum=0.9)
            G = torch.empty(n, n, dtype=torch.float64, device=dev)
            w = torch.zeros(n, device=dev)
            f = max(0, (n - 3) // 2)
            res = {"n": n, "D": D, "dtype": "bf16"}
            res["gram_ms"] = timeit(lambda: K.gram(X, out=G), a.reps)
            # the engine's second, centered pass (rows relative to the medoid row)
            c = K.gram_center(G, n)
            res["gram_centered_ms"] = timeit(lambda: K.gram(X, out=G, center=c), a.reps)
            res["weights_krum_ms"] = timeit(lambda: K.robust_weights(G, "krum", n, f=f, w_out=w), a.reps)
            res["weights_geomed_ms"] = timeit(lambda: K.robust_weights(G, "geomed", n, iters=8, w_out=w), a.reps)
            lo, cnt = K.sorted_range("median", n)
            res["median_sgd_ms"] = timeit(lambda: K.agg_update(
                X, combine="sorted", lo=lo, cnt=cnt, opt=opt, master=master, s1=mom, param_out=p), a.reps)
            lo2, cnt2 = K.sorted_range("trimmed_mean", n, f if 2 * f < n else 0)
            res["trimmed_sgd_ms"] = timeit(lambda: K.agg_update(
                X, combine="sorted", lo=lo2, cnt=cnt2, opt=opt, master=master, s1=mom, param_out=p), a.reps)
            K.robust_weights(G, "krum", n, f=f, w_out=w)
            res["krum_sgd_ms"] = timeit(lambda: K.agg_update(
                X, combine="weighted", w=w, opt=opt, master=master, s1=mom, param_out=p), a.reps)
            wm = torch.full((n,), 1.0 / n, device=dev)
            res["mean_sgd_ms"] = timeit(lambda: K.agg_update(
                X, combine="weighted", w=wm, opt=opt, master=master, s1=mom, param_out=p), a.reps)
            # bytes that must move (HBM): X rows read, master+momentum read+write, params write
            state = D * (4 + 4) * 2 + D * 2
            gbs = lambda byt, ms: round(byt / (ms * 1e-3) / 1e9, 1)
            res["gram_GBps"] = gbs(n * D * 2, res["gram_ms"])
            res["gram_centered_GBps"] = gbs(n * D * 2, res["gram_centered_ms"])
            res["median_sgd_GBps"] = gbs(n * D * 2 + state, res["median_sgd_ms"])
            res["trimmed_sgd_GBps"] = gbs(n * D * 2 + state, res["trimmed_sgd_ms"])
            res["krum_sgd_GBps"] = gbs(D * 2 + state, res["krum_sgd_ms"])
            res["mean_sgd_GBps"] = gbs(n * D * 2 + state, res["mean_sgd_ms"])
            g2 = res["gram_ms"] + res["gram_centered_ms"]   # both Gram passes (engine default)
            res["krum_total_ms"] = round(g2 + res["weights_krum_ms"] + res["krum_sgd_ms"], 4)
            res["geomed_total_ms"] = round(g2 + res["weights_geomed_ms"] + res["mean_sgd_ms"], 4)
            if not a.no_torch:
                Xf = X
                res["torch_median_ms"] = timeit(lambda: torch.median(Xf, dim=0), max(3, a.reps // 4))
                res["torch_sort_ms"] = timeit(lambda: torch.sort(Xf, dim=0), max(3, a.reps // 4))
                res["torch_gram_ms"] = timeit(lambda: (Xf.float() @ Xf.float().t()), max(3, a.reps // 4))
            for k in list(res):
                if isinstance(res[k], float):
                    res[k] = round(res[k], 4)
            line = json.dumps(res)
            print(line, flush=True)
            if a.json_out:
                with open(a.json_out, "a") as fh:
                    fh.write(line + "\n")
            del X


if __name__ == "__main__":
    main()
