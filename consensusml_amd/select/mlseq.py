"""MLSeq-style count classifiers with repeated-CV tuning (C31, `VikasP/AML.R:154-364`).

The reference builds a DESeq dataset from the top-100-variance DEG counts (+1), splits 70/30 and
calls ``MLSeq::classify`` with: svmRadial and pam (on deseq-vst / deseq-rlog), PLDA / PLDA2 /
NBLDA (discrete, ``normalize = "deseq"``), voomDLDA / voomNSC (voom), and the boosting trio
LogitBoost / blackboost / deepboost (on deseq-rlog); ``selectedGenes`` of each fit goes to CSV
(`VikasP/DEG_plda.csv` etc.). This module provides the same method names behind one
``classify(counts, y, method, ...)`` entry point:

  preprocessing  ``deseq_size_factors`` (median of ratios), ``vst`` (parametric-dispersion
                 variance-stabilising transform), ``rlog`` (closed-form regularised log: per-sample
                 log fold changes shrunk toward the gene mean with an empirical-Bayes prior)
  classifiers    ``SVMRadial`` (SMO SVC, sigma by the kernlab ``sigest`` median heuristic, C grid
                 2^(k-3)), ``PAM`` / ``VoomNSC`` (shrunken centroids, threshold grid),
                 ``PLDA`` (rho grid) / ``PLDA2`` (power-transformed counts, PoiClaClu
                 ``FindBestTransform``), ``NBLDA`` (negative-binomial LDA, moment dispersions),
                 ``VoomDLDA``, ``LogitBoost`` (Friedman additive logistic with stumps),
                 ``BlackBoost`` (L2 gradient boosting of binomial deviance with regression trees,
                 nu = 0.1), ``DeepBoost`` (capacity-penalised boosting over tree depths 1..d)
  tuning         repeated stratified k-fold CV over ``tune_length`` grid points; the winning
                 parameter is refit on all training samples (``trained(fit)`` = ``fit.tuning``)
  outputs        ``fit.predict``, ``fit.selected_genes()``, ``confusion_matrix_stats`` (caret's
                 sensitivity / specificity / accuracy with a positive class)

Numbers are parity-unpinned against MLSeq (R is not available); the tests check the statistical
behaviour (separating a planted signal, sparsity of the selected sets, CV determinism).
Samples x genes tensors throughout; everything runs on the tensors' device.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .stats import DLDA, NSC, voom_transform
from .svm import SVC, fit_svcs
from .trees import grow_tree

# ============================================================================ preprocessing


def deseq_size_factors(counts: torch.Tensor) -> torch.Tensor:
    """DESeq median-of-ratios size factors (genes with a zero in any sample are excluded)."""
    x = counts.double()
    keep = (x > 0).all(0)
    if not bool(keep.any()):
        return torch.ones(x.shape[0], dtype=torch.float64, device=x.device)
    lx = torch.log(x[:, keep])
    lgm = lx.mean(0)
    return torch.exp((lx - lgm).median(1).values)


def _nb_dispersion_fit(norm: torch.Tensor):
    """Parametric dispersion trend alpha(mu) = a0 + a1/mu by least squares on the per-gene
    moment estimates (DESeq2 ``fitType = "parametric"`` shape, without the GLM iterations)."""
    mu = norm.mean(0).clamp_min(1e-8)
    var = norm.var(0, unbiased=True)
    disp = ((var - mu) / (mu * mu)).clamp_min(1e-8)
    A = torch.stack([torch.ones_like(mu), 1.0 / mu], 1)
    coef = torch.linalg.lstsq(A, disp[:, None]).solution.flatten()
    a0 = float(coef[0].clamp_min(1e-6))
    a1 = float(coef[1].clamp_min(0.0))
    return a0, a1, disp


def vst(counts: torch.Tensor, sf: Optional[torch.Tensor] = None, fit=None) -> torch.Tensor:
    """Variance-stabilising transform for the parametric trend a0 + a1/mu:
    log2((1 + a1 + 2 a0 q + 2 sqrt(a0 q (1 + a1 + a0 q))) / (4 a0)); ``fit`` reuses the training
    trend (like DESeq2's ``dispersionFunction`` frozen on the training set)."""
    x = counts.double()
    sf = deseq_size_factors(x) if sf is None else sf
    q = x / sf[:, None]
    a0, a1, _ = fit if fit is not None else _nb_dispersion_fit(q)
    return torch.log2((1 + a1 + 2 * a0 * q + 2 * torch.sqrt(a0 * q * (1 + a1 + a0 * q))) / (4 * a0))


def _rlog_parts(x: torch.Tensor, sf: torch.Tensor, fit):
    q = x / sf[:, None]
    a0, a1, _ = fit
    lq = torch.log2(q + 0.5)
    mu = q.mean(0, keepdim=True).clamp_min(0.5)
    svar = (1.0 / mu + a0 + a1 / mu) / (math.log(2) ** 2)
    return lq, mu, svar


def rlog_prior_var(counts: torch.Tensor, sf: Optional[torch.Tensor] = None, fit=None) -> float:
    """Variance of the true log fold changes: mean-squared deviation of the well-expressed genes
    (above-median mean) minus their NB sampling variance."""
    x = counts.double()
    sf = deseq_size_factors(x) if sf is None else sf
    fit = fit if fit is not None else _nb_dispersion_fit(x / sf[:, None])
    lq, mu, svar = _rlog_parts(x, sf, fit)
    dev2 = ((lq - lq.mean(0, keepdim=True)) ** 2).mean(0)
    hi = mu.flatten() > mu.flatten().median()
    return float((dev2[hi] - svar.flatten()[hi]).mean().clamp_min(1e-4))


def rlog(counts: torch.Tensor, sf: Optional[torch.Tensor] = None, fit=None,
         prior_var: Optional[float] = None) -> torch.Tensor:
    """Regularised log: log2 normalised counts whose per-sample deviations from the gene mean are
    shrunk by prior_var / (prior_var + sampling variance), the NB sampling variance of a log2
    count being (1/q + alpha(q)) / ln(2)^2 (``rlog_prior_var`` when ``prior_var`` is None)."""
    x = counts.double()
    sf = deseq_size_factors(x) if sf is None else sf
    fit = fit if fit is not None else _nb_dispersion_fit(x / sf[:, None])
    if prior_var is None:
        prior_var = rlog_prior_var(x, sf, fit)
    lq, _, svar = _rlog_parts(x, sf, fit)
    gm = lq.mean(0, keepdim=True)
    return gm + prior_var / (prior_var + svar) * (lq - gm)


# ============================================================================ classifiers


class _Base:
    """fit(counts, y) / predict(counts) / selected_genes(); y is 0/1."""
    param_name = ""

    def selected_genes(self) -> torch.Tensor:
        return torch.arange(self.p_)


class _Transformed(_Base):
    """Continuous classifier on vst / rlog counts (transform frozen on the training set)."""

    def __init__(self, preprocessing: str = "deseq-vst"):
        self.preprocessing = preprocessing

    def _tx(self, counts, train: bool):
        x = counts.double()
        sf = deseq_size_factors(x)
        if train:
            self.fit_ = _nb_dispersion_fit(x / sf[:, None])
        if self.preprocessing == "deseq-rlog":
            if train:
                self.prior_var_ = rlog_prior_var(x, sf, self.fit_)
            return rlog(x, sf, self.fit_, self.prior_var_)
        return vst(x, sf, self.fit_)


class SVMRadial(_Transformed):
    param_name = "C"

    def __init__(self, C: float = 1.0, preprocessing: str = "deseq-vst", sigma=None):
        super().__init__(preprocessing)
        self.C, self.sigma = C, sigma

    @staticmethod
    def sigest(X: torch.Tensor, frac: float = 0.5, seed: int = 0) -> float:
        """kernlab ``sigest``: inverse of the median squared distance of random pairs (scaled data)."""
        n = X.shape[0]
        g = torch.Generator().manual_seed(seed)
        m = max(2, int(frac * n))
        i = torch.randint(0, n, (m,), generator=g).to(X.device)
        j = torch.randint(0, n, (m,), generator=g).to(X.device)
        d2 = ((X[i] - X[j]) ** 2).sum(1)
        d2 = d2[d2 > 0]
        if d2.numel() == 0:
            return 1.0
        qs = torch.quantile(d2, torch.tensor([0.9, 0.5, 0.1], dtype=d2.dtype, device=d2.device))
        return float((1.0 / qs).mean())

    def fit(self, counts, y):
        X = self._tx(counts, True)
        self.p_ = X.shape[1]
        mu, sd = X.mean(0), X.std(0)
        sd = torch.where(sd > 0, sd, torch.ones_like(sd))
        gamma = self.sigma if self.sigma is not None else self.sigest((X - mu) / sd)
        self.svc = SVC("radial", C=self.C, gamma=gamma).fit(X, y)
        return self

    def predict(self, counts):
        return self.svc.predict(self._tx(counts, False))

    @classmethod
    def cv_accuracy(cls, counts, y, folds, grid, preprocessing: str = "deseq-vst",
                    sigma=None) -> Dict[float, float]:
        """Mean CV accuracy per cost in ``grid``: the per-fold transform and sigma are computed
        once per fold, and every (fold, cost) dual problem is solved in ONE batched SMO launch."""
        Xs, ys, Cs, gs, tests = [], [], [], [], []
        for rep in folds:
            for tr, te in rep:
                tr_t = torch.as_tensor(tr, device=counts.device)
                te_t = torch.as_tensor(te, device=counts.device)
                m = cls(1.0, preprocessing, sigma)
                X = m._tx(counts[tr_t], True)
                mu, sd = X.mean(0), X.std(0)
                sd = torch.where(sd > 0, sd, torch.ones_like(sd))
                gamma = sigma if sigma is not None else cls.sigest((X - mu) / sd)
                Xte = m._tx(counts[te_t], False)
                for c in grid:
                    Xs.append(X)
                    ys.append(y[tr_t])
                    Cs.append(c)
                    gs.append(gamma)
                    tests.append((Xte, y[te]))
        models = fit_svcs(Xs, ys, "radial", C=Cs, gamma=gs)
        acc: Dict[float, List[float]] = {c: [] for c in grid}
        for mdl, c, (Xte, yte) in zip(models, Cs, tests):
            acc[c].append(float((mdl.predict(Xte).cpu() == yte.cpu()).float().mean()))
        return {c: float(np.mean(v)) for c, v in acc.items()}


class PAM(_Transformed):
    """pamr nearest shrunken centroids on vst / rlog data (MLSeq method ``pam``)."""
    param_name = "threshold"

    def __init__(self, threshold: float = 1.0, preprocessing: str = "deseq-vst"):
        super().__init__(preprocessing)
        self.threshold = threshold

    def fit(self, counts, y):
        X = self._tx(counts, True)
        self.p_ = X.shape[1]
        self.nsc = NSC(self.threshold).fit(X, y)
        return self

    def predict(self, counts):
        return self.nsc.predict(self._tx(counts, False))

    def selected_genes(self):
        return self.nsc.selected

    @staticmethod
    def max_threshold(X, y) -> float:
        m = NSC(0.0).fit(X, y)
        return float(m.shrunk.abs().max())


class VoomNSC(_Base):
    param_name = "threshold"

    def __init__(self, threshold: float = 1.0):
        self.threshold = threshold

    def fit(self, counts, y):
        self.p_ = counts.shape[1]
        self.nsc = NSC(self.threshold).fit(voom_transform(counts), y)
        return self

    def predict(self, counts):
        return self.nsc.predict(voom_transform(counts))

    def selected_genes(self):
        return self.nsc.selected


class VoomDLDA(_Base):
    def fit(self, counts, y):
        self.p_ = counts.shape[1]
        self.m = DLDA().fit(voom_transform(counts), y)
        return self

    def predict(self, counts):
        return self.m.predict(voom_transform(counts))


def _null_model(x: torch.Tensor, sf_type: str = "deseq"):
    """PoiClaClu NullModel: per-sample size factors s_i (summing to 1 over training samples) and
    expected counts N_ij = s_i * gene total_j."""
    if sf_type == "deseq":
        s = deseq_size_factors(x)
        s = s / s.sum()
    else:
        s = x.sum(1) / x.sum()
    return s, torch.outer(s, x.sum(0))


class PLDA(_Base):
    """Poisson LDA (Witten 2011): d_kj = (X_kj + beta) / (N_kj + beta), soft-thresholded toward 1
    by rho / sqrt(N_kj + beta); selected genes are those with some d_kj != 1."""
    param_name = "rho"

    def __init__(self, rho: float = 0.0, transform: bool = False, alpha: Optional[float] = None,
                 sf_type: str = "deseq", beta: float = 1.0):
        self.rho, self.transform, self.alpha = rho, transform, alpha
        self.sf_type, self.beta = sf_type, beta

    @staticmethod
    def goodness_of_fit(x: torch.Tensor, sf_type: str = "mle") -> float:
        _, N = _null_model(x, sf_type)
        r = (x - N) ** 2 / N
        return float(torch.nan_to_num(r, nan=0.0, posinf=0.0).sum())

    @classmethod
    def find_best_transform(cls, x: torch.Tensor) -> float:
        """PoiClaClu FindBestTransform: the power alpha in seq(.01, 1, len=50) whose Poisson
        goodness-of-fit statistic is closest to its expectation (n-1)(p-1)."""
        n, p = x.shape
        target = (n - 1) * (p - 1)
        alphas = np.linspace(0.01, 1.0, 50)
        gof = [abs(cls.goodness_of_fit(x.double() ** a) - target) for a in alphas]
        return float(alphas[int(np.argmin(gof))])

    def _prep(self, counts):
        x = counts.double()
        return x ** self.alpha_ if self.transform else x

    def fit(self, counts, y):
        self.alpha_ = (self.alpha if self.alpha is not None else
                       self.find_best_transform(counts)) if self.transform else 1.0
        x = self._prep(counts)
        self.p_ = x.shape[1]
        y = y.to(x.device)
        self.classes = torch.unique(y)
        s, N = _null_model(x, self.sf_type)
        self.gene_tot, self.total = x.sum(0), x.sum()
        d = []
        for c in self.classes:
            m = y == c
            num, den = x[m].sum(0) + self.beta, N[m].sum(0) + self.beta
            dk = num / den
            if self.rho > 0:
                dk = 1 + torch.sign(dk - 1) * ((dk - 1).abs() - self.rho / torch.sqrt(den)).clamp_min(0)
            d.append(dk)
        self.d = torch.stack(d)
        self.prior = torch.stack([(y == c).double().mean() for c in self.classes])
        self.train_x_ = x
        return self

    def _test_sf(self, x):
        if self.sf_type == "deseq":   # test size factors against the training geometric means
            keep = (self.train_x_ > 0).all(0) & (x > 0).all(0)
            if bool(keep.any()):
                lgm = torch.log(self.train_x_[:, keep]).mean(0)
                sf = torch.exp((torch.log(x[:, keep]) - lgm).median(1).values)
                sf_tr = deseq_size_factors(self.train_x_)
                return sf / sf_tr.sum()
        return x.sum(1) / self.total

    def decision(self, counts):
        x = self._prep(counts)
        s = self._test_sf(x)
        N = torch.outer(s, self.gene_tot)
        return x @ torch.log(self.d).t() - N @ self.d.t() + torch.log(self.prior)

    def predict(self, counts):
        return self.classes[self.decision(counts).argmax(1)]

    def selected_genes(self):
        return torch.nonzero((self.d != 1).any(0)).flatten()

    def max_rho(self, counts, y) -> float:
        """Smallest rho that shrinks every d_kj to 1 (top of the tuning grid)."""
        m = PLDA(0.0, self.transform, self.alpha, self.sf_type, self.beta).fit(counts, y)
        x = m._prep(counts)
        _, N = _null_model(x, self.sf_type)
        dens = torch.stack([N[y.to(x.device) == c].sum(0) + self.beta for c in m.classes])
        return float(((m.d - 1).abs() * torch.sqrt(dens)).max())


class PLDA2(PLDA):
    """MLSeq ``PLDA2`` = PLDA on power-transformed counts."""

    def __init__(self, rho: float = 0.0, alpha: Optional[float] = None, sf_type: str = "deseq"):
        super().__init__(rho, True, alpha, sf_type)


class NBLDA(_Base):
    """Negative-binomial LDA (Dong et al. 2016): score_k(x) = sum_j x_j log d_kj
    - (x_j + 1/phi_j) log(1 + s g_j d_kj phi_j) + log pi_k with moment-estimated dispersions
    phi_j (pooled within class, shrunk toward their mean by ``shrink``)."""

    def __init__(self, shrink: float = 0.5, beta: float = 1.0):
        self.shrink, self.beta = shrink, beta

    def fit(self, counts, y):
        x = counts.double()
        self.p_ = x.shape[1]
        y = y.to(x.device)
        self.classes = torch.unique(y)
        s, N = _null_model(x, "deseq")
        self.gene_tot = x.sum(0)
        self.sf_tr_ = deseq_size_factors(x)
        self.train_x_ = x
        self.d = torch.stack([(x[y == c].sum(0) + self.beta) / (N[y == c].sum(0) + self.beta)
                              for c in self.classes])
        cls_idx = (y[:, None] == self.classes[None]).long().argmax(1)
        mu = N * self.d[cls_idx]
        resid = ((x - mu) ** 2 - mu) / mu.clamp_min(1e-8) ** 2
        phi = resid.mean(0).clamp_min(1e-8)
        self.phi = (1 - self.shrink) * phi + self.shrink * phi.mean()
        self.prior = torch.stack([(y == c).double().mean() for c in self.classes])
        return self

    def decision(self, counts):
        x = counts.double()
        keep = (self.train_x_ > 0).all(0) & (x > 0).all(0)
        if bool(keep.any()):
            lgm = torch.log(self.train_x_[:, keep]).mean(0)
            s = torch.exp((torch.log(x[:, keep]) - lgm).median(1).values) / self.sf_tr_.sum()
        else:
            s = x.sum(1) / self.train_x_.sum()
        sc = []
        for k in range(len(self.classes)):
            mk = torch.outer(s, self.gene_tot) * self.d[k]
            sc.append((x * torch.log(self.d[k]) - (x + 1 / self.phi) * torch.log1p(mk * self.phi)).sum(1)
                      + torch.log(self.prior[k]))
        return torch.stack(sc, 1)

    def predict(self, counts):
        return self.classes[self.decision(counts).argmax(1)]


class LogitBoost(_Transformed):
    """caTools LogitBoost: Friedman-Hastie-Tibshirani additive logistic regression with decision
    stumps (weighted least-squares fit to the working response each iteration)."""
    param_name = "nIter"

    def __init__(self, nIter: int = 21, preprocessing: str = "deseq-rlog"):
        super().__init__(preprocessing)
        self.nIter = int(nIter)

    def fit(self, counts, y):
        X = self._tx(counts, True).float()
        self.p_ = X.shape[1]
        yy = y.to(X.device).float()
        n = X.shape[0]
        F = torch.zeros(n, device=X.device)
        self.stumps = []
        rows = torch.arange(n, device=X.device)
        for _ in range(self.nIter):
            p = torch.sigmoid(2 * F)
            w = (p * (1 - p)).clamp_min(1e-10)
            z = ((yy - p) / w).clamp(-4, 4)
            # weighted LS stump: g = -w z, h = w -> leaf = sum(w z) / sum(w)
            t = grow_tree(X, -w * z, w, rows, 1, "xgb", 1e-6, 0.0, 1,
                          leaf_value=lambda gg, hh: -gg.sum() / hh.sum().clamp_min(1e-12))
            self.stumps.append(t)
            F = F + 0.5 * t.predict(X)
        return self

    def decision(self, counts):
        X = self._tx(counts, False).float()
        F = torch.zeros(X.shape[0], device=X.device)
        for t in self.stumps:
            F = F + 0.5 * t.predict(X)
        return F

    def predict(self, counts):
        return (self.decision(counts) > 0).long()

    def selected_genes(self):
        return torch.tensor(sorted({f for t in self.stumps for f in t.feature if f >= 0}),
                            dtype=torch.long)


class BlackBoost(_Transformed):
    """mboost ``blackboost`` (family = Binomial): gradient boosting of the binomial deviance with
    regression trees of depth ``maxdepth`` fitted to the negative gradient, step nu = 0.1."""
    param_name = "mstop"

    def __init__(self, mstop: int = 50, maxdepth: int = 2, nu: float = 0.1,
                 preprocessing: str = "deseq-rlog"):
        super().__init__(preprocessing)
        self.mstop, self.maxdepth, self.nu = int(mstop), maxdepth, nu

    def fit(self, counts, y):
        X = self._tx(counts, True).float()
        self.p_ = X.shape[1]
        yy = y.to(X.device).float()
        n = X.shape[0]
        pbar = float(yy.mean().clamp(1e-3, 1 - 1e-3))
        self.offset = 0.5 * math.log(pbar / (1 - pbar))    # mboost Binomial offset (half log-odds)
        F = torch.full((n,), self.offset, device=X.device)
        ones = torch.ones(n, device=X.device)
        rows = torch.arange(n, device=X.device)
        self.trees = []
        ytil = 2 * yy - 1
        for _ in range(self.mstop):
            ngrad = 2 * ytil / (1 + torch.exp(2 * ytil * F))   # negative gradient of Binomial()
            t = grow_tree(X, -ngrad, ones, rows, self.maxdepth, "xgb", 0.0, 1.0, 2,
                          leaf_value=lambda gg, hh: -gg.sum() / hh.sum())
            self.trees.append(t)
            F = F + self.nu * t.predict(X)
        return self

    def decision(self, counts):
        X = self._tx(counts, False).float()
        F = torch.full((X.shape[0],), self.offset, device=X.device)
        for t in self.trees:
            F = F + self.nu * t.predict(X)
        return F

    def predict(self, counts):
        return (self.decision(counts) > 0).long()

    def selected_genes(self):
        return torch.tensor(sorted({f for t in self.trees for f in t.feature if f >= 0}),
                            dtype=torch.long)


class DeepBoost(_Transformed):
    """DeepBoost (Cortes, Mohri & Syed 2014), exponential loss: each round grows one weighted
    classification tree per depth 1..tree_depth on the current distribution, scores it by its
    edge minus the capacity penalty Lambda_d = lambda * r_d + beta with
    r_d = sqrt(2^(d+1) log(2p + 2) / n) (the Rademacher bound of depth-d trees over p features),
    and adds the best one with the penalised closed-form step."""
    param_name = "num_iter"

    def __init__(self, num_iter: int = 10, tree_depth: int = 3, beta: float = 0.0,
                 lam: float = 0.05, preprocessing: str = "deseq-rlog"):
        super().__init__(preprocessing)
        self.num_iter, self.tree_depth, self.beta, self.lam = int(num_iter), tree_depth, beta, lam

    def fit(self, counts, y):
        X = self._tx(counts, True).float()
        n, p = X.shape
        self.p_ = p
        ys = (2 * y.to(X.device).float() - 1)
        w = torch.full((n,), 1.0 / n, device=X.device)
        rows = torch.arange(n, device=X.device)
        self.ensemble = []
        F = torch.zeros(n, device=X.device)
        for _ in range(self.num_iter):
            best = None
            for d in range(1, self.tree_depth + 1):
                t = grow_tree(X, -w * ys, w, rows, d, "xgb", 1e-9, 0.0, 1,
                              leaf_value=lambda gg, hh: 1.0 if float(-gg.sum()) >= 0 else -1.0)
                h = t.predict(X)
                edge = float((w * ys * h).sum())
                pen = self.lam * math.sqrt(2 ** (d + 1) * math.log(2 * p + 2) / n) + self.beta
                score = abs(edge) - pen
                if best is None or score > best[0]:
                    best = (score, t, edge, pen, h)
            score, t, edge, pen, h = best
            if score <= 0:
                break
            eps_m = (1 - abs(edge)) / 2                       # weighted error of +-h
            a = 0.5 * math.log(max((1 - eps_m) - pen / 2, 1e-12) / max(eps_m + pen / 2, 1e-12))
            a = math.copysign(max(a, 0.0), edge)
            self.ensemble.append((a, t))
            F = F + a * h
            w = torch.exp(-ys * F)
            w = w / w.sum()
        return self

    def decision(self, counts):
        X = self._tx(counts, False).float()
        F = torch.zeros(X.shape[0], device=X.device)
        for a, t in self.ensemble:
            F = F + a * t.predict(X)
        return F

    def predict(self, counts):
        return (self.decision(counts) > 0).long()

    def selected_genes(self):
        return torch.tensor(sorted({f for _, t in self.ensemble for f in t.feature if f >= 0}),
                            dtype=torch.long)


# ============================================================================ CV + classify

METHODS = {
    "svmRadial": SVMRadial, "pam": PAM, "voomNSC": VoomNSC, "voomDLDA": VoomDLDA,
    "PLDA": PLDA, "PLDA2": PLDA2, "NBLDA": NBLDA, "LogitBoost": LogitBoost,
    "blackboost": BlackBoost, "deepboost": DeepBoost,
}


def repeated_stratified_folds(y: torch.Tensor, number: int, repeats: int, seed: int):
    """caret ``repeatedcv`` folds: per repeat, each class is shuffled and dealt round-robin."""
    y = y.cpu().numpy()
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(repeats):
        fold = np.empty(len(y), dtype=np.int64)
        for c in np.unique(y):
            idx = np.nonzero(y == c)[0]
            rng.shuffle(idx)
            fold[idx] = np.arange(len(idx)) % number
        out.append([(np.nonzero(fold != k)[0], np.nonzero(fold == k)[0]) for k in range(number)])
    return out


def _grid(method: str, counts: torch.Tensor, y: torch.Tensor, tune_length: int, kw) -> List:
    if method == "svmRadial":
        return [2.0 ** (k - 2) for k in range(tune_length)]            # caret: 0.25, 0.5, 1, ...
    if method in ("pam", "voomNSC"):
        X = (voom_transform(counts) if method == "voomNSC" else
             PAM(preprocessing=kw.get("preprocessing", "deseq-vst"))._tx(counts, True))
        top = PAM.max_threshold(X, y)
        return list(np.linspace(0.0, top, tune_length + 1)[:-1])     # exclude "no genes left"
    if method in ("PLDA", "PLDA2"):
        top = METHODS[method](**kw).max_rho(counts, y)
        return list(np.linspace(0.0, top, tune_length + 1)[:-1])
    if method == "LogitBoost":
        return [11 + 10 * k for k in range(tune_length)]
    if method == "blackboost":
        return [50 * (k + 1) for k in range(tune_length)]
    if method == "deepboost":
        return [5 * (k + 1) for k in range(tune_length)]
    return [None]


@dataclass
class MLSeqFit:
    method: str
    model: object
    best: object
    tuning: Dict[object, float] = field(default_factory=dict)    # param -> mean CV accuracy

    def predict(self, counts: torch.Tensor) -> torch.Tensor:
        return self.model.predict(counts)

    def selected_genes(self, names: Optional[Sequence[str]] = None):
        idx = self.model.selected_genes()
        return [names[i] for i in idx.tolist()] if names is not None else idx


def _make(method, param, kw):
    cls = METHODS[method]
    if param is None or not cls.param_name:
        return cls(**kw)
    return cls(**{cls.param_name: param}, **kw)


def classify(counts: torch.Tensor, y: torch.Tensor, method: str, number: int = 5,
             repeats: int = 1, tune_length: int = 10, seed: int = 2128, **kw) -> MLSeqFit:
    """MLSeq ``classify``: tune the method's parameter by repeated stratified CV accuracy (ties ->
    the first grid value, i.e. the least regularised), then refit on all samples."""
    if method not in METHODS:
        raise ValueError(f"unknown method {method}; one of {sorted(METHODS)}")
    y = y.long()
    grid = _grid(method, counts, y, tune_length, kw)
    tuning: Dict[object, float] = {}
    if len(grid) > 1:
        folds = repeated_stratified_folds(y, number, repeats, seed)
        if method == "svmRadial":
            tuning = SVMRadial.cv_accuracy(counts, y, folds, grid,
                                           kw.get("preprocessing", "deseq-vst"), kw.get("sigma"))
        for g in (grid if method != "svmRadial" else []):
            accs = []
            for rep in folds:
                for tr, te in rep:
                    tr_t = torch.as_tensor(tr, device=counts.device)
                    te_t = torch.as_tensor(te, device=counts.device)
                    m = _make(method, g, kw).fit(counts[tr_t], y[tr_t])
                    accs.append(float((m.predict(counts[te_t]).cpu() == y[te].cpu()).float().mean()))
            tuning[g] = float(np.mean(accs))
        best = max(grid, key=lambda g: (tuning[g], -grid.index(g)))
    else:
        best = grid[0]
    return MLSeqFit(method, _make(method, best, kw).fit(counts, y), best, tuning)


def confusion_matrix_stats(pred: torch.Tensor, actual: torch.Tensor, positive: int = 1):
    """caret ``confusionMatrix(table(pred, actual), positive=)``: sensitivity, specificity,
    accuracy, PPV / NPV and balanced accuracy."""
    p = pred.cpu().long() == positive
    a = actual.cpu().long() == positive
    tp, tn = int((p & a).sum()), int((~p & ~a).sum())
    fp, fn = int((p & ~a).sum()), int((~p & a).sum())

    def div(x, z):
        return x / z if z else float("nan")
    sens, spec = div(tp, tp + fn), div(tn, tn + fp)
    return {"table": [[tp, fp], [fn, tn]], "sensitivity": sens, "specificity": spec,
            "accuracy": div(tp + tn, tp + tn + fp + fn), "ppv": div(tp, tp + fp),
            "npv": div(tn, tn + fn), "balanced_accuracy": (sens + spec) / 2}
