"""Reference-capability kernels on the GPU: the tree split search of csrc/kernels/tree_hist.hip
against the torch formulation (select/hist_trees._split_search_torch) on the same inputs, and a
whole histogram forest / boosting fit on the GPU (kernel path) against the CPU (torch path)."""
import pytest
import torch

from consensusml_amd.select import hist_trees as HT

pytestmark = pytest.mark.gpu


def _level_inputs(cuda, T, L, n, p, kk, B, crit, seed):
    g = torch.Generator().manual_seed(seed)
    Xb = torch.randint(0, B, (n, p), generator=g, dtype=torch.uint8)
    local = torch.randint(0, L, (T, n), generator=g)
    alive = torch.rand(T, n, generator=g) > 0.2
    if crit == "gini":
        w = torch.randint(0, 3, (T, n), generator=g).float()        # bootstrap counts
        y = torch.randint(0, 2, (n,), generator=g).float()
        stat = torch.stack([w, w * y[None]], -1)
        alive = alive & (w > 0)
    else:
        gr = torch.randn(T, n, generator=g)
        h = torch.rand(T, n, generator=g) * 0.25 + 0.01
        stat = torch.stack([gr, h], -1)
    feats = torch.stack([torch.randperm(p, generator=g)[:kk] for _ in range(T * L)]).view(T, L, kk)
    tt = torch.arange(T)
    key = (tt[:, None] * L + local).view(-1)
    tot = torch.zeros(T * L, 2)
    m = alive.view(-1)
    tot.index_add_(0, key[m], stat.view(-1, 2)[m])
    tot = tot.view(T, L, 2)
    return [t.to(cuda) for t in (Xb, local, alive, stat, feats, tot, tt)]


@pytest.mark.parametrize("crit", ["gini", "xgb"])
@pytest.mark.parametrize("T,L,n,p,kk,B", [(3, 1, 93, 200, 14, 64), (5, 8, 61, 37, 37, 16),
                                          (2, 4, 150, 500, 100, 64)])
def test_split_search_kernel_matches_torch(cuda, crit, T, L, n, p, kk, B):
    from consensusml_amd.ops.native import lib
    Xb, local, alive, stat, feats, tot, tt = _level_inputs(cuda, T, L, n, p, kk, B, crit, T * n)
    best_r, j_r, b_r = HT._split_search_torch(Xb, stat, feats, local, alive, tot, tt, L, kk, B,
                                              crit, 1.0, 1.0 if crit == "xgb" else 0.0)
    nl = torch.where(alive, local, torch.full_like(local, -1)).int()
    best, j, b = lib().split_search(Xb, nl, stat.float(), feats.int(), tot, B,
                                    0 if crit == "gini" else 1, 1.0, 1.0 if crit == "xgb" else 0.0)
    fin = torch.isfinite(best_r)
    assert torch.equal(fin, torch.isfinite(best))
    torch.testing.assert_close(best[fin], best_r[fin], rtol=1e-4, atol=1e-4)
    if crit == "gini":   # integer statistics: identical sums, identical winners
        assert torch.equal(j.long()[fin], j_r[fin]) and torch.equal(b.long()[fin], b_r[fin])


@pytest.mark.parametrize("kind", ["forest", "boost"])
def test_hist_ensemble_gpu_matches_cpu(cuda, kind):
    torch.manual_seed(0)
    n, p = 120, 60
    X = torch.randn(n, p)
    y = ((X[:, 0] + 0.5 * X[:, 3] - X[:, 7]) > 0).long()
    mk = (lambda: HT.HistForest(n_estimators=64, max_depth=5, seed=3)) if kind == "forest" else \
        (lambda: HT.HistBoost(n_estimators=20, max_depth=3, seed=3))
    cpu = mk().fit(X, y)
    gpu = mk().fit(X.to(cuda), y.to(cuda))
    pc = cpu.predict_proba(X)
    pg = gpu.predict_proba(X.to(cuda)).cpu()
    assert (pc - pg).abs().mean().item() < 0.05
    ic, ig = cpu.feature_importances_.double(), gpu.feature_importances_.double().cpu()
    assert torch.corrcoef(torch.stack([ic, ig]))[0, 1].item() > 0.9
    acc = (gpu.predict(X.to(cuda)).cpu() == y).float().mean().item()
    assert acc > 0.85


@pytest.mark.parametrize("intercept", [False, True])
@pytest.mark.parametrize("alpha", [1.0, 0.5])
def test_fista_gpu_kernels_match_cpu(cuda, intercept, alpha):
    """csrc/kernels/lasso_prox.hip (residual, prox / restart / momentum) reproduces the CPU
    FISTA path: same problems (LOOCV-style masks x lambda grid), same optimum."""
    from consensusml_amd.select.lasso import fista_logistic
    g = torch.Generator().manual_seed(2)
    n, p = 40, 300
    X = torch.randn(n, p, generator=g)
    y = (X[:, :5].sum(1) + 0.3 * torch.randn(n, generator=g) > 0).float()
    lams = torch.tensor([0.2, 0.05, 0.02, 0.005]).repeat(3)
    masks = torch.ones(n, lams.numel())
    for k in range(3):                      # three held-out samples
        masks[k, 4 * k:4 * k + 4] = 0
    bc, b0c, itc, _ = fista_logistic(X, y, lams, masks, intercept=intercept, alpha=alpha,
                                     max_iter=2000, tol=1e-7)
    bg, b0g, itg, _ = fista_logistic(X.to(cuda), y.to(cuda), lams, masks.to(cuda),
                                     intercept=intercept, alpha=alpha, max_iter=2000, tol=1e-7)
    torch.testing.assert_close(bg.cpu(), bc, rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(b0g.cpu(), b0c, rtol=2e-3, atol=2e-3)
    # identical support on clearly nonzero coefficients
    sig = bc.abs() > 1e-2
    assert torch.equal(sig, bg.cpu().abs() > 1e-2) or (sig ^ (bg.cpu().abs() > 1e-2)).sum() <= 2


def test_exact_forest_gpu(cuda):
    """ExactForest (exact thresholds, in-kernel candidate sampling): fits the training rows,
    ranks the informative features first like the CPU exact RandomForest, the same total
    MeanDecreaseGini per tree, and a symmetric proximity matrix with a unit diagonal."""
    from consensusml_amd.select.hist_trees import ExactForest
    from consensusml_amd.select.trees import RandomForest
    g = torch.Generator().manual_seed(5)
    n, p = 93, 400
    X = torch.randn(n, p, generator=g)
    y = (X[:, :3].sum(1) > 0).long()
    ef = ExactForest(400, seed=2).fit(X.to(cuda), y.to(cuda))
    assert ef.exact
    assert (ef.predict(X.to(cuda)).cpu() == y).float().mean() > 0.95
    imp = ef.mean_decrease_gini
    assert {0, 1, 2} <= set(torch.topk(imp, 6).indices.tolist())
    rf = RandomForest(100, seed=2).fit(X, y)
    assert {0, 1, 2} <= set(torch.topk(rf.mean_decrease_gini, 6).indices.tolist())
    # fully grown trees on the same rows: the Gini decreases add up to about the same per tree
    ratio = float(imp.sum() / rf.mean_decrease_gini.sum())
    assert 0.8 < ratio < 1.25, ratio
    P = ef.proximity(X.to(cuda)).cpu()
    assert torch.allclose(P, P.t()) and torch.allclose(P.diag(), torch.ones(n))
