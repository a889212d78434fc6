"""C30 cohort summary and C31 voom classifiers — CPU."""
import torch

from consensusml_amd.select.data import synthetic_cohort
from consensusml_amd.select.mlseq import PLDA, VoomDLDA, VoomNSC
from consensusml_amd.select.stats import cohort_summary


def test_cohort_summary_chisq():
    es = synthetic_cohort(200, 60, seed=4)
    s = cohort_summary(es.col_data)
    assert s["n"] == 60 and sum(s["classes"].values()) == 60
    assert 0.0 <= s["gender"]["p_value"] <= 1.0 and s["age"]["df"] == 1


def test_voom_classifiers_separate_strong_signal():
    es = synthetic_cohort(400, 80, n_signal=40, effect=2.0, seed=6)
    X = es.assays["counts"].t()
    y = torch.tensor(es.col_data.low_risk.values)
    for m in (VoomDLDA(), VoomNSC(0.5), PLDA()):
        m.fit(X[:60], y[:60])
        assert (m.predict(X[60:]) == y[60:]).float().mean() > 0.85, type(m).__name__
    nsc = VoomNSC(2.0).fit(X[:60], y[:60])
    assert 0 < nsc.selected_genes().numel() < 400
