#!/usr/bin/env python3
"""Column-by-column comparison of a ``python -m consensusml_amd.select --rdata ...`` run's
``standouttable.csv`` with the reference's saved ``standouttable.csv``
(composite_code/rnotebook/data/standouttable.csv). Prints a markdown table: Pearson / Spearman
correlation, nonzero counts and top-50 overlap per model column, with notes on the reference's
own known defects that make some columns incomparable.

  python tools/reference_parity_report.py out/standouttable.csv [--ref PATH]
"""
import argparse

import numpy as np
import pandas as pd
from scipy.stats import spearmanr

NOTES = {
    "lasso_coef_rep": "reference keeps 1 coefficient per rep (loop bug SEA:787); compared on "
                      "its single gene",
    "svm2_weights": "reference svm2 == svm1 (weights taken before the refit, SEA:155)",
    "svm4_weights": "reference radial 'weights' are meaningless (SEA:155); ours: none",
    "svm3_weights": "reference radial 'weights' are meaningless (SEA:155); ours: none",
    "rfnb": "stochastic (randomForest vs our CART forest, different RNG)",
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ours")
    ap.add_argument("--ref", default="/root/reference/composite_code/rnotebook/data/standouttable.csv")
    a = ap.parse_args()
    ours = pd.read_csv(a.ours, index_col=0)
    ref = pd.read_csv(a.ref, index_col=0).loc[ours.index]
    print("| column | pearson | spearman | nonzero ours / ref | top-50 overlap | note |")
    print("|---|---|---|---|---|---|")
    for c in ref.columns:
        if c not in ours.columns or ref[c].dtype == object:
            continue
        x, y = ours[c].to_numpy(float), ref[c].to_numpy(float)
        note = next((v for k, v in NOTES.items() if c.startswith(k)), "")
        if np.isnan(x).all():
            print(f"| {c} | - | - | - | - | {note} |")
            continue
        if c.startswith("lasso_coef_rep"):
            nzr = np.nonzero(y)[0]
            same = ", ".join(f"{ours.index[i]}: ours {x[i]:.4f} ref {y[i]:.4f}" for i in nzr)
            print(f"| {c} | - | - | {np.count_nonzero(x)} / {len(nzr)} | - | {note}: {same} |")
            continue
        p = np.corrcoef(x, y)[0, 1] if x.std() > 0 and y.std() > 0 else float("nan")
        s = spearmanr(x, y).correlation
        top = len(set(np.argsort(-np.abs(x))[:50]) & set(np.argsort(-np.abs(y))[:50]))
        print(f"| {c} | {p:.6f} | {s:.4f} | {np.count_nonzero(x)} / {np.count_nonzero(y)} | "
              f"{top} | {note} |")


if __name__ == "__main__":
    main()
