"""Reference-capability module (select/) vs scikit-learn / scipy golden values on small
synthetic p >> n data. CPU."""
import numpy as np
import pandas as pd
import pytest
import torch

from consensusml_amd.select import consensus as C
from consensusml_amd.select import data as D
from consensusml_amd.select import filters as F
from consensusml_amd.select import metrics as M
from consensusml_amd.select import normalize as N
from consensusml_amd.select import stats as S
from consensusml_amd.select.lasso import cv_lasso, l1_logistic_sklearn_like, run_lasso
from consensusml_amd.select.svm import SVC, run_svm, weight_quantile_genes
from consensusml_amd.select.trees import GradientBoostedTrees, RandomForest


def _data(n=80, p=200, seed=0):
    g = np.random.default_rng(seed)
    X = g.standard_normal((n, p)).astype(np.float32)
    w = np.zeros(p)
    w[:5] = 2.0
    y = (X @ w + g.standard_normal(n) > 0).astype(np.int64)
    return torch.tensor(X), torch.tensor(y)


@pytest.mark.parametrize("C_", [0.05, 0.5])
def test_l1_logistic_matches_sklearn(C_):
    from sklearn.linear_model import LogisticRegression
    X, y = _data()
    sk = LogisticRegression(penalty="l1", C=C_, solver="liblinear", fit_intercept=False,
                            tol=1e-10, max_iter=100000).fit(X.numpy(), y.numpy())
    b, _ = l1_logistic_sklearn_like(X, y, C_, fit_intercept=False, max_iter=20000, tol=1e-9)
    assert np.abs(sk.coef_[0] - b.numpy()).max() < 1e-4
    assert ((sk.coef_[0] != 0) == (b.numpy() != 0)).all()


def test_cv_lasso_lambda_rule():
    X, y = _data(60, 100)
    cv = cv_lasso(X, y, nfolds=None)
    i = np.argmin(cv["cvm"])
    assert cv["lambda_min"] >= cv["lambda"][i] - 1e-12
    assert cv["cvm"][list(cv["lambda"]).index(cv["lambda_min"])] == cv["cvm"].min()
    assert cv["lambda_1se"] >= cv["lambda_min"]


def test_run_lasso_result_list():
    X, y = _data(90, 150)
    genes = [f"g{i}" for i in range(150)]
    r = run_lasso(X, y, genes, list(range(60)), list(range(60, 90)))
    for k in ["training_set", "testing_set", "contrast", "train_fit", "cv_fit",
              "confusion_matrix", "test_error", "final_model", "nonzero_coef", "seed"]:
        assert k in r
    assert r["test_error"] < 0.3
    assert any(g in r["nonzero_coef"] for g in ["g0", "g1", "g2", "g3", "g4"])


def test_svm_matches_libsvm():
    from sklearn.svm import SVC as SK
    X, y = _data(70, 120, 1)
    Xn = X.double().numpy()
    Xs = (Xn - Xn.mean(0)) / Xn.std(0, ddof=1)
    for kern, skk in (("linear", "linear"), ("radial", "rbf")):
        sk = SK(kernel=skk, C=1.0, gamma=1.0 / 120, tol=1e-6).fit(Xs, y.numpy())
        m = SVC(kern, tol=1e-6).fit(X, y)
        np.testing.assert_allclose(m.decision_function(X).numpy(), sk.decision_function(Xs),
                                   atol=1e-4)


def test_run_svm_weightfilt():
    X, y = _data(80, 60, 2)
    r = run_svm(50, "linear", X[:50], y[:50], X[50:], y[50:], 0.5)
    assert len(r["features_used"]) == 30
    assert r["weightsvect"] is not None and (r["weightsvect"] != 0).sum() <= 30
    r2 = run_svm(50, "radial", X[:50], y[:50], X[50:], y[50:])
    assert r2["weightsvect"] is None
    q = weight_quantile_genes(torch.randn(1000), [str(i) for i in range(1000)])
    assert len(q["high"][0.01]) == 10


def test_random_forest_vs_sklearn_importance_rank():
    from sklearn.ensemble import RandomForestClassifier
    g = np.random.default_rng(0)
    X = g.standard_normal((150, 40)).astype(np.float32)
    y = ((X[:, 0] + 0.8 * X[:, 1]) > 0).astype(np.int64)
    rf = RandomForest(60, seed=1).fit(torch.tensor(X), torch.tensor(y))
    sk = RandomForestClassifier(200, random_state=0).fit(X, y)
    assert set(torch.topk(rf.feature_importances_, 2).indices.tolist()) == \
        set(np.argsort(-sk.feature_importances_)[:2].tolist())
    P = rf.proximity(torch.tensor(X[:10]))
    assert torch.allclose(torch.diagonal(P), torch.ones(10))


def test_gbt_learns_and_importance():
    X, y = _data(120, 50, 3)
    m = GradientBoostedTrees(60, 0.3, 3).fit(X[:90], y[:90])
    p = m.predict_proba(X[90:])[:, 1]
    assert ((p > 0.5).long() == y[90:]).float().mean() > 0.7
    assert int(torch.argmax(m.feature_importances_)) < 5


def test_tmm_and_logcpm():
    es = D.synthetic_cohort(n_genes=300, n_samples=20, seed=1)
    cnt = es.assays["counts"]
    f = N.tmm_factors(cnt)
    assert abs(float(torch.log(f).mean())) < 1e-9
    # scaling one library leaves TMM factors (x lib size) invariant up to the geometric-mean norm
    cnt2 = cnt.clone()
    cnt2[:, 0] *= 3
    f2 = N.tmm_factors(cnt2)
    assert torch.allclose(f2[1:] / f2[1], f[1:] / f[1], rtol=1e-6)
    lc = N.log_cpm(cnt)
    lib = cnt.double().sum(0)
    prior = lib / lib.mean()
    ref = torch.log2((cnt.double() + prior) / (lib + 2 * prior) * 1e6)
    assert torch.allclose(lc, ref)
    keep = N.filter_by_cpm(cnt, 1.0, 5)
    assert keep.dtype == torch.bool and keep.sum() > 0


def test_voom_de_finds_signal():
    from consensusml_amd.select.de import voom_de, bh_adjust
    es = D.synthetic_cohort(n_genes=800, n_samples=60, n_signal=30, effect=2.0, seed=3)
    y = es.col_data["low_risk"].tolist()
    deg = voom_de(es.assays["counts"], y, es.genes)
    sig = set(es.row_data.index[es.row_data.signal])
    assert len(deg) > 10
    assert len(set(deg.index) & sig) / len(deg) > 0.8
    p = np.array([0.01, 0.04, 0.03, 0.2])
    from scipy.stats import false_discovery_control
    np.testing.assert_allclose(bh_adjust(p), false_discovery_control(p))


def test_spearman_matches_scipy():
    from scipy.stats import spearmanr
    g = np.random.default_rng(0)
    X = g.integers(0, 5, (30, 6)).astype(np.float64)   # ties
    r = S.spearman(torch.tensor(X)).numpy()
    np.testing.assert_allclose(r, spearmanr(X).correlation, atol=1e-10)


def test_kmeans_glmboost_chisq_dlda():
    g = np.random.default_rng(0)
    X = np.concatenate([g.normal(0, 0.1, (20, 2)), g.normal(3, 0.1, (20, 2))])
    lab, Cc, wss = S.kmeans(torch.tensor(X), 2, nstart=5)
    assert len(set(lab[:20].tolist())) == 1 and lab[0] != lab[-1]
    Xr = torch.tensor(g.standard_normal((100, 10)))
    yr = 3 * Xr[:, 2] - 2 * Xr[:, 7] + 0.01 * torch.tensor(g.standard_normal(100))
    b0, beta = S.glmboost(Xr, yr, mstop=500, nu=0.1)
    assert torch.topk(beta.abs(), 2).indices.sort().values.tolist() == [2, 7]
    res = S.chisq_test(np.array([[10, 20], [20, 10]]))
    assert 0 < res["p_value"] < 0.05
    yc = torch.tensor([0] * 20 + [1] * 20)
    d = S.DLDA().fit(torch.tensor(X), yc)
    assert (d.predict(torch.tensor(X)) == yc).all()
    nsc = S.NSC(delta=0.5).fit(torch.tensor(X), yc)
    assert (nsc.predict(torch.tensor(X)) == yc).all()


def test_metrics_reference_definitions():
    y = torch.tensor([1, 1, 1, 0, 0, 0, 0, 1])
    p = torch.tensor([1, 0, 1, 0, 1, 0, 0, 1])
    m = M.binary_metrics(y, p)
    assert m["tpr"] == 3 / 4 and m["tnr"] == 3 / 4
    assert abs(m["fdr"] - (1 - 3 / 4)) < 1e-12 and abs(m["for"] - (1 - 3 / 4)) < 1e-12
    from sklearn.metrics import log_loss, roc_auc_score
    pr = torch.tensor([0.9, 0.2, 0.8, 0.3, 0.6, 0.1, 0.4, 0.7])
    assert abs(M.log_loss(y, pr) - log_loss(y.numpy(), pr.numpy())) < 1e-6
    assert abs(M.auc(y, pr) - roc_auc_score(y.numpy(), pr.numpy())) < 1e-9


def test_standard_table_consensus_and_csv(tmp_path):
    genes = [f"g{i}" for i in range(6)]
    t = C.StandardTable(genes, pd.DataFrame({"logFC": np.arange(6.0)}, index=genes))
    t.add("lasso_coef_rep1", {"g0": 0.5, "g2": -0.1})
    t.add("svm1_weights", np.array([0.3, 0.0, 0.2, 0.0, 0.0, 0.01]))
    t.add("xg1_imp", np.array([0.7, 0.0, 0.0, 0.3, 0.0, 0.0]))
    t.add_consensus()
    assert t.df.loc["g0", "consensus_votes"] == 3
    assert t.df.loc["g1", "consensus_votes"] == 0
    p = tmp_path / "standouttable.csv"
    t.to_csv(str(p))
    back = C.StandardTable.read_csv(str(p))
    assert list(back.df.columns) == list(t.df.columns)
    np.testing.assert_allclose(back.df["svm1_weights"].to_numpy(), t.df["svm1_weights"].to_numpy())
    sets = {k: C.selected(t.df[k]) for k in t.runs}
    inter = C.intersections(sets)
    assert inter["lasso_coef_rep1&svm1_weights&xg1_imp"] == {"g0"}
    mt = C.membership_table(sets)
    assert mt.loc["g0", "n_models"] == 3


def test_outlier_model_detection():
    g = np.random.default_rng(0)
    base = g.random(200)
    X = torch.tensor(np.stack([base + 0.01 * g.random(200) for _ in range(5)] + [g.random(200)]),
                     dtype=torch.float32)
    r = C.outlier_models(X, f=1)
    assert not bool(r["kept"][5])


def test_data_plumbing(tmp_path):
    files = []
    for k in range(3):
        p = tmp_path / f"s{k}.htseq.counts"
        p.write_text("ENSG1.1\t5\nENSG2.3\t7\n__no_feature\t9\n")
        files.append(str(p))
    m = D.concat_count_files(files)
    assert m.shape == (2, 3)
    manifest = pd.DataFrame({"project.project_id": ["TARGET-AML", "TARGET-NBL"],
                             "entity_submitter_id": ["TARGET-20-PAAAAA-09A-01R",
                                                     "TARGET-30-PBBBBB-01A-01R"]})
    clinical = pd.DataFrame({"TARGET USI": ["TARGET-20-PAAAAA"], "Risk group": ["Low"]})
    mc = D.merge_manifest_clinical(manifest, clinical, "TARGET-AML")
    assert len(mc) == 1
    assay = pd.DataFrame({"gene": ["ENSG1", "ENSG2"], "TARGET.20.PAAAAA.09A.01R": [1.0, 2.0]})
    at = D.transpose_assay(assay)
    merged = D.merge_assay_clinical(at, mc)
    assert merged.columns[1] == "Diagnostic ID" and merged["Diagnostic ID"].iloc[0] == "09A"
    oh = D.one_hot_like_train(pd.Series(["a", "c"]), ["a", "b"], "x")
    assert oh.values.tolist() == [[1, 0], [0, 0]]
    keep = D.select_primary_samples(["TARGET.20.PA1.09A.01R", "TARGET.20.PA2.14A.01R",
                                     "TARGET.21.PA3.09A.01R"])
    assert keep == [0]
    es = D.synthetic_cohort(100, 12)
    es.save(str(tmp_path / "es"))
    es2 = D.ExpressionSet.load(str(tmp_path / "es"))
    assert torch.equal(es.assays["counts"], es2.assays["counts"]) and es2.genes == es.genes
    tr, te = F.seeded_split(es.samples)
    assert len(tr) == 8 and not set(tr) & set(te)
    X = torch.randn(40, 30)
    yy = torch.tensor([0, 1] * 20)
    cols = F.variance_filter(X, yy, 5)
    assert 5 <= cols.numel() <= 10
    a, b, h = F.holdout_split(100)
    assert len(h) == 20 and len(set(a) | set(b) | set(h)) == 100


def test_pipeline_end_to_end(tmp_path):
    from consensusml_amd.select.pipeline import consensus_pipeline
    es = D.synthetic_cohort(n_genes=600, n_samples=60, n_signal=30, effect=1.2, seed=5)
    out = consensus_pipeline(es, out_dir=str(tmp_path), lasso_reps=2, rf_trees=(20,),
                             max_genes=120, xgb_configs=({"max_depth": 2, "n_estimators": 2},
                                                         {"max_depth": 6, "n_estimators": 10}))
    assert (tmp_path / "standouttable.csv").exists()
    df = out["table"].df
    for col in ["logFC", "p.adj.bh", "svm1_weights", "lasso_coef_rep1", "rfnb_20_MeanDecNodeImp",
                "xg1_imp", "consensus_votes"]:
        assert col in df.columns
    assert out["performance"]["test_error"].max() < 0.5


def test_plots(tmp_path):
    from consensusml_amd.select import plots as P
    g = np.random.default_rng(0)
    deg = pd.DataFrame({"logFC": g.normal(0, 2, 200), "p.adj.bh": g.random(200) ** 4},
                       index=[f"g{i}" for i in range(200)])
    P.volcano(deg, str(tmp_path / "v.png"), dpi=50)
    P.heatmap(g.random((20, 12)), str(tmp_path / "h.png"), [f"g{i}" for i in range(20)],
              [0, 1] * 6, dpi=50)
    P.importance_bars(deg["logFC"], str(tmp_path / "b.png"), dpi=50)
    P.rep_performance({"tpr": [0.9, 0.8], "tnr": [0.8, 0.7]}, str(tmp_path / "r.png"), dpi=50)
    P.correlation_density(np.corrcoef(g.random((10, 30))), str(tmp_path / "c.png"), dpi=50)
    assert all((tmp_path / f).stat().st_size > 0 for f in ["v.png", "h.png", "b.png", "r.png", "c.png"])


def test_cpm_filter_strict_fraction_boundary():
    """Limma_Voom_DE_Function.R:27 keeps a gene when rowSums(cpm >= 1) > 0.05 * ncol: at n = 100
    a gene needs 6 expressing samples (5 is not enough); at n = 90 (4.5) 5 suffice."""
    for n, need in ((100, 6), (90, 5), (40, 3)):
        cnt = torch.zeros(3, n, dtype=torch.float64)
        cnt[2, :] = 1e6           # gene 2: every sample (sets library sizes ~1e6)
        cnt[0, :need] = 100.0     # gene 0: exactly `need` samples with CPM >= 1 (~100)
        cnt[1, :need - 1] = 100.0  # gene 1: one fewer
        keep = N.filter_by_cpm(cnt, 1.0, None, 0.05)
        assert keep.tolist() == [True, False, True], (n, keep.tolist())
