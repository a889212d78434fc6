"""Level-synchronous histogram forests / boosting (select/hist_trees.py) — CPU."""
import numpy as np
import torch

from consensusml_amd.select.hist_trees import HistBoost, HistForest, bin_with, quantile_bins


def _easy(n=300, p=100, seed=1):
    g = np.random.default_rng(seed)
    X = g.standard_normal((n, p)).astype(np.float32)
    y = ((X[:, 0] + 0.7 * X[:, 5]) > 0).astype(np.int64)
    return torch.tensor(X), torch.tensor(y)


def test_quantile_bins_monotone():
    X, _ = _easy(200, 8)
    Xb, edges = quantile_bins(X, 16)
    assert Xb.max() <= 15
    # binning is monotone in x and reproduced by bin_with
    for j in range(8):
        o = torch.argsort(X[:, j])
        assert (Xb[o, j][1:] >= Xb[o, j][:-1]).all()
    assert torch.equal(bin_with(X, edges), Xb)


def test_hist_forest_learns_and_ranks_features():
    X, y = _easy()
    f = HistForest(150, 6, seed=3).fit(X[:200], y[:200])
    acc = (f.predict(X[200:]) == y[200:]).float().mean()
    assert acc > 0.75
    assert set(torch.topk(f.feature_importances_, 2).indices.tolist()) == {0, 5}
    assert f.mean_decrease_gini.shape == (100,)


def test_hist_boost_learns():
    X, y = _easy()
    b = HistBoost(60, 0.3, 3, seed=2).fit(X[:200], y[:200])
    p = b.predict_proba(X[200:])[:, 1]
    assert ((p > 0.5).long() == y[200:]).float().mean() > 0.85
    assert set(torch.topk(b.feature_importances_, 2).indices.tolist()) == {0, 5}
    b2 = HistBoost(20, 0.3, 3, colsample=0.5, seed=2).fit(X[:200], y[:200])
    assert torch.isfinite(b2.predict_proba(X[200:])).all()


def test_depth_zero_is_prior():
    X, y = _easy(100, 8)
    f = HistForest(10, 0, seed=0).fit(X, y)
    p = f.predict_proba(X)[:, 1]
    assert torch.allclose(p, p[0].expand_as(p))


def test_rf_and_xgb_resultslists():
    from consensusml_amd.select.trees import rf_resultslist, xgb_resultslist
    torch.manual_seed(0)
    n, p = 80, 12
    X = torch.randn(n, p)
    y = (X[:, 0] + 0.5 * X[:, 1] > 0).long()
    rf = rf_resultslist(X[:60], y[:60], X[60:], y[60:], ntrees=(200, 1000))
    assert set(rf) == {"rf200_results", "rf1k_results"}
    r = rf["rf1k_results"]
    assert int(r["conf_matrix"].sum()) == 20 and r["conf_matrix"].trace() >= 15
    P = r["proximity"]
    assert P.shape == (60, 60) and torch.allclose(P.diagonal(), torch.ones(60))
    assert torch.allclose(P, P.t()) and (P >= 0).all() and (P <= 1).all()
    xg = xgb_resultslist(X[:60], y[:60], X[60:], y[60:])
    df = xg["testperfdf"]
    assert list(df.index) == [f"rep{i}" for i in range(1, 6)]
    assert list(df.columns) == ["mean_err", "tpr", "tnr", "fdr", "for"]
    for i in range(1, 6):
        perf = xg[f"rep{i}"]["performance_testset"]
        assert abs(perf["mean_err"] - df.loc[f"rep{i}", "mean_err"]) < 1e-12
        assert int(perf["confusion_matrix"].sum()) == 20


def test_exact_bins_are_distinct_value_ranks():
    """exact_bins: one bin per distinct value (its rank), edges at the midpoints between
    consecutive distinct values, +inf padding; x <= edge_b <=> bin <= b for any x."""
    from consensusml_amd.select.hist_trees import exact_bins
    g = torch.Generator().manual_seed(3)
    X = torch.randint(0, 7, (40, 5), generator=g).float() * 0.5
    X[:, 4] = torch.randn(40, generator=g)          # 40 distinct values
    Xb, edges, B = exact_bins(X)
    for f in range(5):
        u = torch.unique(X[:, f])
        rank = torch.searchsorted(u, X[:, f])
        assert torch.equal(Xb[:, f].long(), rank)
        k = u.numel()
        torch.testing.assert_close(edges[f, :k - 1], (u[1:] + u[:-1]) / 2)
        assert torch.isinf(edges[f, k - 1:]).all()
    assert B == 40
    t = torch.randn(100, 5, generator=g)
    tb = bin_with(t, edges)
    for f in range(5):
        for b in range(3):
            assert torch.equal(t[:, f] <= edges[f, b], tb[:, f].long() <= b)
    assert exact_bins(torch.randn(300, 2, generator=g), max_bins=128) is None
