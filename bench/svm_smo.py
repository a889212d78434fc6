#!/usr/bin/env python3
"""SVM solve time: host numpy SMO (the round-1 path) vs the batched GPU SMO kernel, on the
reference's problem shape (n = 97 training samples x 1984 genes, linear and radial) and on a
batch of CV fits (MLSeq svmRadial: 5 folds x 3 repeats x 8 costs = 120 problems).

  python bench/svm_smo.py
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from consensusml_amd.select.svm import SVC, fit_svcs
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    n, p = 97, 1984
    X = torch.randn(n, p, generator=g, dtype=torch.float64)
    y = (X[:, :20].sum(1) + 3 * torch.randn(n, generator=g, dtype=torch.float64) > 0).long()
    rows = []
    for kern in ("linear", "radial"):
        for label, d in (("host numpy SMO", torch.device("cpu")), ("GPU SMO kernel", dev)):
            Xd, yd = X.to(d), y.to(d)
            SVC(kern).fit(Xd, yd)
            if d.type == "cuda":
                torch.cuda.synchronize()
            t = time.perf_counter()
            reps = 5
            for _ in range(reps):
                m = SVC(kern).fit(Xd, yd)
            if d.type == "cuda":
                torch.cuda.synchronize()
            rows.append({"case": f"single fit {kern} n={n} p={p}", "impl": label,
                         "ms": round((time.perf_counter() - t) / reps * 1e3, 3),
                         "iters": getattr(m, "n_iter_", None), "n_sv": int(m.support_.numel())})
    # CV grid: 120 problems of ~78 samples
    folds = []
    for r in range(3):
        perm = torch.randperm(n, generator=torch.Generator().manual_seed(r))
        for k in range(5):
            tr = torch.cat([perm[:k * n // 5], perm[(k + 1) * n // 5:]])
            folds.append(tr)
    Cs = [2.0 ** (c - 3) for c in range(8)]
    probs = [(f, c) for f in folds for c in Cs]
    for label, d in (("host numpy SMO", torch.device("cpu")), ("GPU SMO kernel (1 launch)", dev)):
        Xd, yd = X.to(d), y.to(d)
        t = time.perf_counter()
        fit_svcs([Xd[f] for f, _ in probs], [yd[f] for f, _ in probs], "radial",
                 C=[c for _, c in probs])
        if d.type == "cuda":
            torch.cuda.synchronize()
        rows.append({"case": f"CV grid radial: {len(probs)} fits of n~{len(folds[0])}",
                     "impl": label, "ms": round((time.perf_counter() - t) * 1e3, 3)})
    for r in rows:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
