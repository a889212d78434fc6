#!/usr/bin/env python3
"""Write tests/fixtures/reference_subset.npz from the reference's saved data (read with the
data-only R reader; nothing in the files is executed): the analysis container's log-CPM matrix
(1984 DEGs x 137 samples), labels, train/test split, gene ids, the standard-table columns the
parity tests compare against (rfnb_*, xg*_imp, svm1_weights, DE statistics) and lasso rep 1's
lambda.min / test error / nonzero coefficients. GPU boxes have no /root/reference; with this
fixture tests/test_reference_rdata_parity.py runs there too.

  python tools/make_ref_fixture.py [--ref /root/reference/composite_code/rnotebook/data]
"""
import argparse
import os
import sys

import numpy as np
import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

COLS = ["logFC", "AveExpr", "t", "p.unadj", "p.adj.bh", "b", "svm1_weights",
        "rfnb_2k_MeanDecNodeImp", "rfnb_5k_MeanDecNodeImp", "rfnb_10k_MeanDecNodeImp",
        "xg1_imp", "xg2_imp", "xg3_imp", "xg4_imp", "xg5_imp"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference/composite_code/rnotebook/data")
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "fixtures", "reference_subset.npz"))
    a = ap.parse_args()
    from consensusml_amd.select import rdata as R
    from consensusml_amd.select.data import ExpressionSet
    es = ExpressionSet.from_rdata(os.path.join(a.ref, "sesetfilt_degseahack_targetaml.rda"))
    cd = es.col_data
    split = cd["exptset.seahack"].to_numpy()
    st = pd.read_csv(os.path.join(a.ref, "standouttable.csv"), index_col=0).loc[es.genes]
    rl = R.read_rdata(os.path.join(a.ref, "lasso_resultslist.rda"))["lasso.resultslist"][0]
    nz = rl["nonzero.coef"]
    np.savez_compressed(
        a.out,
        X=es.assays["logcpm"].t().contiguous().numpy().astype(np.float32),
        y=pd.to_numeric(cd["deg.risk"]).to_numpy().astype(np.int64),
        train=np.where(split == "train")[0], test=np.where(split == "test")[0],
        genes=np.array(list(es.genes), dtype="U32"),
        st_cols=np.array(COLS, dtype="U32"),
        st=np.stack([st[c].to_numpy(dtype=np.float64) for c in COLS], 1),
        lasso_lambda_min=np.float64(rl["cv.fit"]["lambda.min"].values[0]),
        lasso_test_error=np.float64(rl["test.error"].values[0]),
        lasso_genes=np.array(list(R.names(nz)), dtype="U32"),
        lasso_coef=np.asarray(nz.values, dtype=np.float64))
    print("wrote", a.out, os.path.getsize(a.out), "bytes")


if __name__ == "__main__":
    main()
