#!/usr/bin/env python3
"""The reference's only published timings, re-measured on MI355X (BASELINE.md "Throughput /
timing"): sklearn RandomForest fit, 300 trees, depth 3, ~73 samples x {1,496; 21,404; 3,110}
genes = 0.2 s / 0.6 s / 0.3 s on a developer laptop CPU (`scripts/model_walkthrough.ipynb:195`,
`:1639`, `:1563`). Same shapes, synthetic data, ``HistForest`` (level-synchronous histogram
forest, all trees of a level in one batched pass) on the GPU; fit time includes binning and is
synchronised. Also times the full glmnet-style LOOCV lasso path (93 x 1,984, 100 lambdas, the
reference's `runLasso` shape) for context (no reference number). One JSON line per row.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ROWS = [("rf300_d3_1496genes", 1496, 0.2), ("rf300_d3_21404genes", 21404, 0.6),
        ("rf300_d3_3110genes", 3110, 0.3)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    from consensusml_amd.select.hist_trees import HistForest
    from consensusml_amd.select.lasso import cv_lasso, lasso_path
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    g = np.random.default_rng(8)
    out = []
    for name, p, ref_s in ROWS:
        X = torch.tensor(g.standard_normal((73, p)).astype(np.float32), device=dev)
        y = torch.tensor((g.random(73) < 0.45).astype(np.int64), device=dev)
        HistForest(300, 3, seed=8).fit(X, y)          # warm-up (allocator, kernels)
        sync()
        ts = []
        for _ in range(a.reps):
            t = time.perf_counter()
            HistForest(300, 3, seed=8).fit(X, y)
            sync()
            ts.append(time.perf_counter() - t)
        ts.sort()
        med = ts[len(ts) // 2]
        out.append({"row": name, "device": str(dev), "fit_s": round(med, 4),
                    "reference_s": ref_s, "speedup_vs_reference": round(ref_s / med, 2),
                    "note": "reference: sklearn RF n_jobs=1 on an unspecified laptop CPU"})
    X = torch.tensor(g.standard_normal((93, 1984)).astype(np.float32), device=dev)
    y = torch.tensor((g.random(93) < 0.45).astype(np.int64), device=dev)
    cv_lasso(X[:20], y[:20])
    sync()
    t = time.perf_counter()
    cv = cv_lasso(X, y)
    lasso_path(X, y)
    sync()
    out.append({"row": "lasso_loocv_path_93x1984_100lambda", "device": str(dev),
                "fit_s": round(time.perf_counter() - t, 4), "reference_s": None,
                "lambda_min": cv["lambda_min"],
                "note": "93 folds x 100 lambdas solved as one batched FISTA problem"})
    for r in out:
        line = json.dumps(r)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "a") as fh:
                fh.write(line + "\n")


if __name__ == "__main__":
    main()
