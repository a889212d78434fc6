"""Classical statistics and the smaller classifiers of the reference (C28, C30, C31, C32, C33).

* ``spearman``             rank-transform + Pearson Gram on the device (C28, 1984 x 1984 from
                           137 samples at `cml_targetaml_seanalysis.Rmd:889-1016`).
* ``chisq_test``           Pearson chi-square of a contingency table (C30, `...:455-470`).
* ``kmeans``               Lloyd with k-means++ seeding and nstart restarts (C33,
                           `BuieRProj/KM_WHATEVER.Rmd:151-187`).
* ``glmboost``             component-wise L2 boosting regression (C32, mlr ``regr.glmboost``,
                           `Ryan/Feature_selection_GLMTrain_WT_TARGET.R:56-64`).
* ``DLDA`` / ``NSC``        diagonal LDA and nearest shrunken centroids: the base estimators of
                           the MLSeq wrappers in ``select/mlseq.py`` (C31, ``voomDLDA`` / ``pam``
                           / ``voomNSC`` at `VikasP/AML.R:174-264`; Poisson LDA lives there too).
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Sequence

import numpy as np
import torch
from scipy import stats as sps


def rank_columns(X: torch.Tensor) -> torch.Tensor:
    """Average-tie ranks of every column (samples x features)."""
    X = X.double()
    n = X.shape[0]
    order = torch.argsort(X, dim=0)
    ranks = torch.empty_like(X)
    ar = torch.arange(1, n + 1, dtype=torch.float64, device=X.device).view(-1, 1).expand_as(X)
    ranks.scatter_(0, order, ar.contiguous())
    # average ties: group equal values per column
    s = torch.gather(X, 0, order)
    r_sorted = torch.gather(ranks, 0, order)
    out = ranks.clone()
    tie = s[1:] == s[:-1]
    if bool(tie.any()):
        for j in torch.nonzero(tie.any(0)).flatten().tolist():
            col = s[:, j]
            _, inv, cnt = torch.unique_consecutive(col, return_inverse=True, return_counts=True)
            ends = torch.cumsum(cnt, 0).double()
            avg = (ends - cnt.double() + 1 + ends) / 2
            out[order[:, j], j] = avg[inv]
    return out


def pearson(X: torch.Tensor) -> torch.Tensor:
    Z = X.double() - X.double().mean(0)
    Z = Z / Z.norm(dim=0).clamp_min(1e-300)
    return Z.t() @ Z


def spearman(X: torch.Tensor) -> torch.Tensor:
    """Feature x feature Spearman correlation of a samples x features matrix."""
    return pearson(rank_columns(X))


def chisq_test(table: np.ndarray, correct: bool = True) -> Dict[str, float]:
    """R ``chisq.test`` (Yates continuity correction for 2x2 by default)."""
    t = np.asarray(table, dtype=np.float64)
    chi2, p, dof, _ = sps.chi2_contingency(t, correction=correct and t.shape == (2, 2))
    return {"statistic": float(chi2), "p_value": float(p), "df": int(dof)}


def kmeans(X: torch.Tensor, k: int, nstart: int = 25, iters: int = 100, seed: int = 1000):
    """Returns (labels, centers, total within-cluster SS) of the best of ``nstart`` runs."""
    X = X.double()
    n = X.shape[0]
    g = torch.Generator().manual_seed(seed)
    best = None
    for _ in range(nstart):
        c = [int(torch.randint(0, n, (1,), generator=g))]
        for _ in range(1, k):
            d2 = torch.cdist(X, X[c]).pow(2).min(1).values
            pr = (d2 / d2.sum().clamp_min(1e-300)).cpu()
            c.append(int(torch.multinomial(pr, 1, generator=g)))
        C = X[c].clone()
        lab = None
        for _ in range(iters):
            nl = torch.cdist(X, C).argmin(1)
            if lab is not None and torch.equal(nl, lab):
                break
            lab = nl
            for j in range(k):
                m = lab == j
                if bool(m.any()):
                    C[j] = X[m].mean(0)
        wss = float(((X - C[lab]) ** 2).sum())
        if best is None or wss < best[2]:
            best = (lab, C, wss)
    return best


def glmboost(X: torch.Tensor, y: torch.Tensor, mstop: int = 100, nu: float = 0.1):
    """Component-wise L2 boosting (mboost::glmboost, centred covariates). Returns the intercept
    and the coefficient vector (non-selected features stay 0)."""
    X = X.double()
    y = y.double()
    mu = X.mean(0)
    Xc = X - mu
    ss = (Xc * Xc).sum(0).clamp_min(1e-300)
    f0 = y.mean()
    r = y - f0
    beta = torch.zeros(X.shape[1], dtype=torch.float64, device=X.device)
    for _ in range(mstop):
        b = (Xc.t() @ r) / ss
        rss = ((r[:, None] - Xc * b) ** 2).sum(0)
        j = int(torch.argmin(rss))
        beta[j] += nu * b[j]
        r = r - nu * b[j] * Xc[:, j]
    return float(f0 - (mu * beta).sum()), beta


class DLDA:
    """Diagonal LDA on (voom-like log) expression: class means, pooled per-gene variance."""

    def fit(self, X, y):
        X = X.double()
        self.classes = torch.unique(y)
        self.means = torch.stack([X[y == c].mean(0) for c in self.classes])
        res = torch.cat([X[y == c] - X[y == c].mean(0) for c in self.classes])
        self.var = (res ** 2).sum(0) / max(X.shape[0] - len(self.classes), 1) + 1e-8
        self.prior = torch.stack([(y == c).double().mean() for c in self.classes])
        return self

    def decision(self, X):
        X = X.double()
        d = ((X[:, None, :] - self.means[None]) ** 2 / self.var).sum(-1)
        return -0.5 * d + torch.log(self.prior)

    def predict(self, X):
        return self.classes[self.decision(X).argmax(1)]


class NSC(DLDA):
    """Nearest shrunken centroids (PAM): soft-threshold standardised centroid offsets by
    ``delta``; ``selected`` genes are those with a non-zero shrunken offset in some class."""

    def __init__(self, delta: float = 1.0):
        self.delta = delta

    def fit(self, X, y):
        super().fit(X, y)
        X = X.double()
        n = X.shape[0]
        overall = X.mean(0)
        s = torch.sqrt(self.var)
        s0 = s.median()
        K = len(self.classes)
        self.shrunk = []
        for k, c in enumerate(self.classes):
            nk = (y == c).sum().double()
            mk = math.sqrt(1.0 / nk + 1.0 / n)
            d = (self.means[k] - overall) / (mk * (s + s0))
            ds = torch.sign(d) * (d.abs() - self.delta).clamp_min(0)
            self.shrunk.append(ds)
            self.means[k] = overall + mk * (s + s0) * ds
        self.shrunk = torch.stack(self.shrunk)
        self.var = (s + s0) ** 2
        self.selected = torch.nonzero((self.shrunk != 0).any(0)).flatten()
        return self


def voom_transform(counts: torch.Tensor) -> torch.Tensor:
    """log2-CPM with 0.5 offsets (the voom expression scale used by MLSeq's voomDLDA / voomNSC),
    samples x genes counts in, samples x genes out."""
    x = counts.double()
    lib = x.sum(1, keepdim=True)
    return torch.log2((x + 0.5) / (lib + 1.0) * 1e6)


def cohort_summary(col_data, label: str = "low_risk", covariates=("gender", "age"),
                   age_cut: Optional[float] = None) -> Dict[str, object]:
    """Cohort table and balance tests (C30, `cml_targetaml_seanalysis.Rmd:422-474`): class counts,
    per-covariate contingency tables vs the label and chi-square p values (numeric covariates
    are split at the median, or at ``age_cut``)."""
    import pandas as pd
    out: Dict[str, object] = {"n": int(len(col_data)),
                              "classes": col_data[label].value_counts().to_dict()}
    for cov in covariates:
        if cov not in col_data:
            continue
        v = col_data[cov]
        if np.issubdtype(v.dtype, np.number):
            # R: ifelse(age >= median(age), "old", "young")  (SEA:463)
            cut = age_cut if age_cut is not None else float(v.median())
            v = (v >= cut).map({True: f">={cut:g}", False: f"<{cut:g}"})
        tab = pd.crosstab(v, col_data[label])
        out[cov] = {"table": tab.to_dict(), **chisq_test(tab.to_numpy())}
    return out
