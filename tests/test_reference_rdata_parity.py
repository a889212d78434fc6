"""Parity against the reference's OWN saved results, read with the data-only R reader
(``consensusml_amd.select.rdata``) from /root/reference (read-only):

* the analysis container ``sesetfilt_degseahack_targetaml.rda`` (1984 DEGs x 137 samples,
  `composite_code/rnotebook/cml_targetaml_seanalysis.Rmd:409-415`) and its DE statistics vs the
  saved ``standouttable.csv``;
* linear SVM weights vs ``standouttable.csv`` ``svm1_weights`` (e1071/libsvm, `...Rmd:647-690`);
* lasso rep 1 (LOOCV lambda.min, test error, selected genes) vs ``lasso_resultslist.rda``
  (glmnet, `...Rmd:68-123`, `:728-778`);
* XGBoost gain importance vs ``standouttable.csv`` ``xg1_imp..xg5_imp`` (`...Rmd:1164-1263`);
* random-forest Gini importance vs ``rf_noboost_2k5k10ktrees_allresultslist.rda``
  (`...Rmd:1022-1091`), judged against the reference's own seed-to-seed spread.
"""
import os

import numpy as np
import pandas as pd
import pytest
import torch

def _ref_dir() -> str:
    """The reference's saved data: /root/reference (here), or a copy under <repo>/refdata (GPU
    boxes have no /root/reference; the copy is git-ignored), or $CML_REFERENCE_DATA."""
    env = os.environ.get("CML_REFERENCE_DATA")
    if env:
        return env
    ref = "/root/reference/composite_code/rnotebook/data"
    if os.path.exists(ref):
        return ref
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "refdata")


REF = _ref_dir()
SE = os.path.join(REF, "sesetfilt_degseahack_targetaml.rda")
STAND = os.path.join(REF, "standouttable.csv")
# derived, data-only subset (tools/make_ref_fixture.py): what the model-parity tests need, so they
# also run on GPU boxes without /root/reference
FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures",
                       "reference_subset.npz")
HAVE_RDA = os.path.exists(SE)

pytestmark = pytest.mark.skipif(not (HAVE_RDA or os.path.exists(FIXTURE)),
                                reason="reference files not present")
needs_rda = pytest.mark.skipif(not HAVE_RDA, reason="needs the reference's .rda files")


@pytest.fixture(scope="module")
def ref():
    if HAVE_RDA:
        from consensusml_amd.select.data import ExpressionSet
        es = ExpressionSet.from_rdata(SE)
        cd = es.col_data
        tr = np.where(cd["exptset.seahack"].to_numpy() == "train")[0]
        te = np.where(cd["exptset.seahack"].to_numpy() == "test")[0]
        y = torch.tensor(pd.to_numeric(cd["deg.risk"]).to_numpy(), dtype=torch.long)
        X = es.assays["logcpm"].t().contiguous()
        st = pd.read_csv(STAND, index_col=0).loc[es.genes]
        return {"es": es, "X": X, "y": y, "tr": tr, "te": te, "st": st, "genes": list(es.genes),
                "source": "rda"}
    z = np.load(FIXTURE)                        # allow_pickle=False (default): arrays only
    genes = [str(g) for g in z["genes"]]
    st = pd.DataFrame(z["st"], index=genes, columns=[str(c) for c in z["st_cols"]])
    return {"es": None, "X": torch.from_numpy(z["X"]), "y": torch.from_numpy(z["y"]),
            "tr": z["train"], "te": z["test"], "st": st, "genes": genes, "fixture": z,
            "source": "fixture"}


def test_fixture_matches_rda():
    """The committed fixture is exactly what the data-only reader extracts from the reference."""
    if not (HAVE_RDA and os.path.exists(FIXTURE)):
        pytest.skip("needs both the .rda files and the fixture")
    from consensusml_amd.select.data import ExpressionSet
    es = ExpressionSet.from_rdata(SE)
    z = np.load(FIXTURE)
    np.testing.assert_array_equal(z["X"], es.assays["logcpm"].t().contiguous().numpy()
                                  .astype(np.float32))
    assert [str(g) for g in z["genes"]] == list(es.genes)


@needs_rda
def test_rdata_container_matches_reference(ref):
    es, st = ref["es"], ref["st"]
    assert es.shape == (1984, 137)                                  # SEA:454 "1984 137"
    assert (len(ref["tr"]), len(ref["te"])) == (93, 44)
    assert int((ref["y"] == 1).sum()) == 77 and int((ref["y"] == 0).sum()) == 60
    for c in ("logFC", "AveExpr", "t", "p.unadj", "p.adj.bh", "b"):
        np.testing.assert_allclose(es.row_data[c].to_numpy(), st[c].to_numpy(), rtol=1e-6)
    assert list(es.row_data["hgnc_symbol"].fillna("")) == list(st["hgnc_symbol"].fillna(""))


@needs_rda
def test_rdata_reader_objects():
    from consensusml_amd.select import rdata as R
    ann = R.read_rdata(os.path.join(REF, "dfens_v95hg38_bmart.rda"))["dfens"]
    df = R.as_frame(ann)
    assert len(df) == 18100 and {"hgnc_symbol", "start", "end", "strand"} <= set(df.columns)
    lasso = R.read_rdata(os.path.join(REF, "lasso_resultslist.rda"))["lasso.resultslist"]
    assert len(lasso) == 15
    assert lasso[0].keys() == ["training.set", "testing.set", "contrast", "train.fit", "cv.fit",
                               "confusionMatrix", "test.error", "final.model", "nonzero.coef",
                               "seed"]
    # strict mode refuses the functions / environments inside Bioconductor containers
    with pytest.raises(R.RDataError):
        R.read_rdata(SE, strict=True)


def test_svm1_weights_parity(ref):
    from consensusml_amd.select.svm import run_svm
    X, y, tr, te = ref["X"], ref["y"], ref["tr"], ref["te"]
    r = run_svm(50, "linear", X[tr], y[tr], X[te], y[te], None, ref["genes"])
    w = r["weightsvect"].numpy()
    w_ref = ref["st"]["svm1_weights"].to_numpy()
    assert np.corrcoef(w, w_ref)[0, 1] > 0.9999
    np.testing.assert_allclose(w, w_ref, rtol=5e-3, atol=2e-5)
    top = lambda v: set(np.argsort(-np.abs(v))[:50])   # noqa: E731
    assert len(top(w) & top(w_ref)) >= 48


def test_lasso_rep1_parity(ref):
    from consensusml_amd.select.lasso import run_lasso
    if ref["source"] == "rda":
        from consensusml_amd.select import rdata as R
        rl = R.read_rdata(os.path.join(REF, "lasso_resultslist.rda"))["lasso.resultslist"][0]
        lmin_ref = float(rl["cv.fit"]["lambda.min"].values[0])
        terr_ref = float(rl["test.error"].values[0])
        nz = rl["nonzero.coef"]
        ref_coef = dict(zip(R.names(nz), nz.values))
    else:
        z = ref["fixture"]
        lmin_ref, terr_ref = float(z["lasso_lambda_min"]), float(z["lasso_test_error"])
        ref_coef = dict(zip([str(g) for g in z["lasso_genes"]], z["lasso_coef"]))
    res = run_lasso(ref["X"].float(), ref["y"], ref["genes"], ref["tr"], ref["te"], seed=2019)
    assert abs(res["cv_fit"]["lambda_min"] - lmin_ref) / lmin_ref < 1e-6       # 0.1630
    assert abs(res["test_error"] - terr_ref) < 1e-6                            # 3 / 44
    ours = res["nonzero_coef"]
    assert set(ref_coef) == set(ours)                                          # 13 genes
    a = np.array([ours[g] for g in ref_coef])
    b = np.array(list(ref_coef.values()))
    assert np.corrcoef(a, b)[0, 1] > 0.9999
    # per coefficient vs glmnet's refit (`...seanalysis.Rmd:110-115`): ours is the exact optimum
    # (objective 0.32552073 vs glmnet's 0.32552075, glmnet stops at thresh = 1e-7), so the
    # tolerance is glmnet's own convergence error: < 1 % relative on every coefficient above
    # 1e-3, and < 5e-5 absolute on the one at the selection boundary (2.75e-4)
    big = np.abs(b) > 1e-3
    np.testing.assert_allclose(a[big], b[big], rtol=1e-2)
    np.testing.assert_allclose(a[~big], b[~big], atol=5e-5)


def test_xgb_importance_parity(ref):
    from consensusml_amd.select.trees import GradientBoostedTrees
    X, y, tr = ref["X"], ref["y"], ref["tr"]
    for i, (depth, rounds) in enumerate([(2, 2), (50, 2), (50, 50)]):
        g = GradientBoostedTrees(rounds, 1.0, depth).fit(X[tr], y[tr])
        imp = g.importance.numpy()
        imp = imp / imp.sum()
        r = ref["st"][f"xg{i + 1}_imp"].to_numpy()
        # exact greedy split search with XGBoost's arithmetic (double sums, float loss change,
        # kRtEps, lower-feature tie-break: select/trees.py _best_split) reproduces all three
        # reference runs, the depth-50 ones included (round 5: 4 of 7 / 7 of 13 shared genes)
        np.testing.assert_allclose(imp, r, atol=1e-6)
        assert set(np.nonzero(imp)[0]) == set(np.nonzero(r)[0])


def test_rf_importance_parity(ref):
    """randomForest is stochastic: our exact-CART forest's Gini importance must agree with the
    reference's 2k-tree run about as well as the reference's own 10k-tree run does (Spearman
    0.77, top-50 overlap 43 between rf2k and rf10k)."""
    from scipy.stats import spearmanr
    from consensusml_amd.select.trees import RandomForest
    imp2k = ref["st"]["rfnb_2k_MeanDecNodeImp"].to_numpy()
    if ref["source"] == "rda":
        from consensusml_amd.select import rdata as R
        RF = R.read_rdata(os.path.join(REF, "rf_noboost_2k5k10ktrees_allresultslist.rda"))
        rf = RF["rf.returnlist"]
        imp_rda = R.as_array(rf["rf2k.results"]["fitmodel"]["importance"]).ravel()
        np.testing.assert_allclose(imp_rda, imp2k, rtol=1e-9)
    X, y, tr = ref["X"], ref["y"], ref["tr"]
    m = RandomForest(2000, seed=20).fit(X[tr], y[tr])     # the reference's rf2k size
    ours = m.mean_decrease_gini.numpy()
    # achieved: 0.656 vs rf2k, 0.760 vs rf10k (the reference's own rf2k vs rf10k: 0.77)
    assert spearmanr(ours, imp2k).correlation > 0.62
    assert spearmanr(ours, ref["st"]["rfnb_10k_MeanDecNodeImp"].to_numpy()).correlation > 0.72
    top = lambda v: set(np.argsort(-v)[:50])   # noqa: E731
    assert len(top(ours) & top(imp2k)) >= 36


@needs_rda
def test_pipeline_on_reference_container_with_resume(tmp_path, monkeypatch):
    """The reference analysis run from its own DEG container, interrupted after the SVM stage
    and resumed: the finished stage is not recomputed (its result list and table columns are
    reloaded), and the outputs keep the reference's standard-table layout."""
    from consensusml_amd.select import pipeline as P
    from consensusml_amd.select import results as RS
    from consensusml_amd.select.data import ExpressionSet
    es = ExpressionSet.from_rdata(SE)
    kw = dict(label_col="deg.risk", split_col="exptset.seahack", deg_from_container=True,
              out_dir=str(tmp_path), lasso_reps=3, rf_trees=(100,), max_genes=400,
              xgb_configs=P.REF_XGB[:2])

    def boom(*a, **k):
        raise RuntimeError("killed")
    monkeypatch.setattr(P, "iterative_exclusion", boom)
    with pytest.raises(RuntimeError, match="killed"):
        P.consensus_pipeline(es, **kw)
    assert RS.exists(str(tmp_path / "results" / "svm4reps_resultslist"))
    saved = pd.read_csv(tmp_path / P.TABLE_FILE, index_col=0)
    assert "svm1_weights" in saved.columns and "lasso_coef_rep1" not in saved.columns
    monkeypatch.undo()
    monkeypatch.setattr(P, "run_svm", boom)          # must not run again
    out = P.consensus_pipeline(es, resume=True, **kw)
    assert out["resumed_stages"] == ["svm4reps_resultslist"]
    np.testing.assert_allclose(out["table"].df["svm1_weights"].to_numpy(),
                               saved["svm1_weights"].to_numpy())
    svm = RS.load_results(str(tmp_path / "results" / "svm4reps_resultslist"))
    assert set(svm) == {"svm1", "svm2", "svm3", "svm4"}
    assert svm["svm1"]["weightsvect"].shape == (400,) and svm["svm3"]["weightsvect"] is None
    lasso = RS.load_results(str(tmp_path / "results" / "lasso_resultslist"))
    assert set(lasso["rep1"]) >= {"training.set", "testing.set", "cv.fit", "confusionMatrix",
                                  "test.error", "nonzero.coef", "seed"}
    assert len(lasso["rep1"]["training.set"]) == 93
    rf = RS.load_results(str(tmp_path / "results" / "rf_noboost_resultslist"))
    assert rf["rf100.results"]["proximity"].shape == (93, 93)
    header = pd.read_csv(tmp_path / "standouttable.csv", index_col=0, nrows=1).columns.tolist()
    assert header == P.DE_COLUMNS + ["lasso_coef_rep1", "lasso_coef_rep2", "lasso_coef_rep3",
                                     "rfnb_100_MeanDecNodeImp", "svm1_weights", "svm2_weights",
                                     "svm3_weights", "svm4_weights", "xg1_imp", "xg2_imp"]


@pytest.mark.gpu
def test_rf_10k_importance_parity_gpu(ref):
    """The reference's 10k-tree forest (the run with the least seed noise) vs ours at the same
    size on the GPU: Spearman >= 0.85 (the committed full run reached 0.88)."""
    from scipy.stats import spearmanr
    from consensusml_amd.select.trees import RandomForest
    X, y, tr = ref["X"].cuda(), ref["y"].cuda(), ref["tr"]
    m = RandomForest(10000, seed=20).fit(X[tr], y[tr])
    ours = m.mean_decrease_gini.cpu().numpy()
    r = spearmanr(ours, ref["st"]["rfnb_10k_MeanDecNodeImp"].to_numpy()).correlation
    assert r >= 0.85, r
