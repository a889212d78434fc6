"""C31 MLSeq-style classifiers (`VikasP/AML.R:154-364`) — CPU. Parity with MLSeq is unpinned (no R);
these pin the statistical behaviour: planted-signal separation, sparsity of selected genes,
transform properties and deterministic CV."""
import pytest
import torch

from consensusml_amd.select import mlseq as M
from consensusml_amd.select.data import synthetic_cohort


@pytest.fixture(scope="module")
def data():
    es = synthetic_cohort(100, 90, n_signal=15, effect=2.0, seed=11)
    X = es.assays["counts"].t().double() + 1          # the reference adds 1 before DESeq
    y = torch.tensor(es.col_data.low_risk.values).long()
    return X[:63], y[:63], X[63:], y[63:]


def test_size_factors_and_transforms(data):
    X = data[0]
    sf = M.deseq_size_factors(X)
    assert sf.shape == (63,) and (sf > 0).all()
    # doubling a sample doubles its size factor
    X2 = X.clone()
    X2[0] *= 2
    assert torch.isclose(M.deseq_size_factors(X2)[0] / sf[0], torch.tensor(2.0, dtype=torch.float64), rtol=0.05)
    v = M.vst(X)
    r = M.rlog(X)
    assert torch.isfinite(v).all() and torch.isfinite(r).all()
    # vst is monotone in the count; rlog shrinks deviations vs plain log2
    lq = torch.log2(X / sf[:, None] + 0.5)
    assert ((r - r.mean(0)).abs().sum() <= (lq - lq.mean(0)).abs().sum() + 1e-9)


@pytest.mark.parametrize("method", ["svmRadial", "pam", "voomNSC", "voomDLDA", "PLDA", "PLDA2",
                                    "NBLDA", "LogitBoost", "blackboost", "deepboost"])
def test_classify_methods_separate_signal(data, method):
    Xtr, ytr, Xte, yte = data
    fit = M.classify(Xtr, ytr, method, number=3, repeats=1, tune_length=3, seed=2128)
    acc = float((fit.predict(Xte) == yte).float().mean())
    assert acc >= 0.75, (method, acc, fit.best)
    sel = fit.selected_genes()
    assert 0 < sel.numel() <= Xtr.shape[1]
    st = M.confusion_matrix_stats(fit.predict(Xte), yte, positive=1)
    assert abs(st["accuracy"] - acc) < 1e-12


def test_sparse_methods_select_few_genes(data):
    Xtr, ytr = data[0], data[1]
    nsc = M.VoomNSC(threshold=M.PAM.max_threshold(M.voom_transform(Xtr), ytr) * 0.6).fit(Xtr, ytr)
    assert 0 < nsc.selected_genes().numel() < 50
    pl = M.PLDA()
    top = pl.max_rho(Xtr, ytr)
    assert M.PLDA(rho=top * 1.0001).fit(Xtr, ytr).selected_genes().numel() == 0
    assert M.PLDA(rho=0.0).fit(Xtr, ytr).selected_genes().numel() == Xtr.shape[1]


def test_plda2_transform_and_cv_determinism(data):
    Xtr, ytr = data[0], data[1]
    a = M.PLDA.find_best_transform(Xtr)
    assert 0.01 <= a <= 1.0
    f1 = M.classify(Xtr, ytr, "PLDA", number=3, tune_length=4, seed=5)
    f2 = M.classify(Xtr, ytr, "PLDA", number=3, tune_length=4, seed=5)
    assert f1.tuning == f2.tuning and f1.best == f2.best
    folds = M.repeated_stratified_folds(ytr, 5, 2, seed=1)
    assert len(folds) == 2 and all(len(r) == 5 for r in folds)
    for rep in folds:
        te = sorted(i for _, t in rep for i in t.tolist())
        assert te == list(range(len(ytr)))
