"""C-support-vector classification (C23, C33): libsvm-style SMO on a precomputed kernel matrix,
e1071 semantics (``scale=TRUE`` column standardisation, cost 1, radial gamma = 1/p), the primal
weight vector w = sum_i alpha_i y_i x_i, and ``run_svm`` with the weight-filter refit.

Reference: ``runSVM`` (`composite_code/rnotebook/cml_targetaml_seanalysis.Rmd:126-210`). Its
``weightsvect`` is taken BEFORE the weight-filter refit and is meaningless for the radial kernel
(SURVEY.md §4.3); here the weights always come from the model that is returned, and radial
models report ``weights=None``.

The Gram / kernel matrix (n x n, n ~ 100) is one GEMM on the device; SMO itself is a few hundred
O(n) vector steps with libsvm's second-order working-set selection.
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence

import numpy as np
import torch

from .metrics import binary_metrics, roc_curve


def kernel_matrix(A: torch.Tensor, B: torch.Tensor, kind: str, gamma: float) -> torch.Tensor:
    A = A.double()
    B = B.double()
    if kind == "linear":
        return A @ B.t()
    if kind == "radial":
        d2 = (A * A).sum(1, keepdim=True) + (B * B).sum(1)[None] - 2 * A @ B.t()
        return torch.exp(-gamma * d2.clamp_min(0))
    raise ValueError(kind)


def smo(K: np.ndarray, y: np.ndarray, C: float = 1.0, tol: float = 1e-3, max_iter: int = 100000):
    """Dual C-SVC: min 1/2 a^T Q a - e^T a, 0 <= a <= C, y^T a = 0 (Q = y y^T * K).
    Returns (alpha, b) with the decision function sum_i a_i y_i K(x_i, x) + b."""
    n = y.size
    Q = K * np.outer(y, y)
    a = np.zeros(n)
    G = -np.ones(n)                       # gradient of the dual objective
    tau = 1e-12
    for _ in range(max_iter):
        up = ((y > 0) & (a < C)) | ((y < 0) & (a > 0))
        lo = ((y > 0) & (a > 0)) | ((y < 0) & (a < C))
        if not up.any() or not lo.any():
            break
        v = -y * G
        i = np.where(up, v, -np.inf).argmax()
        gmax = v[i]
        gmin = np.where(lo, v, np.inf).min()
        if gmax - gmin < tol:
            break
        # second-order working set selection (libsvm WSS2)
        b_ = gmax - v
        a_ = K[i, i] + np.diag(K) - 2 * y[i] * y * Q[i] * y
        a_ = np.where(a_ > 0, a_, tau)
        cand = lo & (v < gmax)
        obj = np.where(cand, -(b_ * b_) / a_, np.inf)
        j = obj.argmin()
        if not np.isfinite(obj[j]):
            break
        # analytic two-variable update (libsvm)
        if y[i] != y[j]:
            quad = max(Q[i, i] + Q[j, j] + 2 * Q[i, j], tau)
            delta = (-G[i] - G[j]) / quad
            diff = a[i] - a[j]
            ai, aj = a[i] + delta, a[j] + delta
            if diff > 0 and aj < 0:
                aj, ai = 0, diff
            elif diff <= 0 and ai < 0:
                ai, aj = 0, -diff
            if diff > 0 and ai > C:
                ai, aj = C, C - diff
            elif diff <= 0 and aj > C:
                aj, ai = C, C + diff
        else:
            quad = max(Q[i, i] + Q[j, j] - 2 * Q[i, j], tau)
            delta = (G[i] - G[j]) / quad
            s = a[i] + a[j]
            ai, aj = a[i] - delta, a[j] + delta
            if s > C and ai > C:
                ai, aj = C, s - C
            elif s <= C and aj < 0:
                aj, ai = 0, s
            if s > C and aj > C:
                aj, ai = C, s - C
            elif s <= C and ai < 0:
                ai, aj = 0, s
        dai, daj = ai - a[i], aj - a[j]
        a[i], a[j] = ai, aj
        G += Q[:, i] * dai + Q[:, j] * daj
    # bias: average over free SVs (libsvm's rho)
    free = (a > 1e-12) & (a < C - 1e-12)
    yG = y * G
    if free.any():
        rho = yG[free].mean()
    else:
        up = ((y > 0) & (a < C)) | ((y < 0) & (a > 0))
        lo = ((y > 0) & (a > 0)) | ((y < 0) & (a < C))
        ub = yG[lo].min() if lo.any() else 0.0
        lb = yG[up].max() if up.any() else 0.0
        rho = (ub + lb) / 2
    return a, -rho


class SVC:
    def __init__(self, kernel: str = "linear", C: float = 1.0, gamma: Optional[float] = None,
                 scale: bool = True, tol: float = 1e-3):
        self.kernel, self.C, self.gamma, self.scale, self.tol = kernel, C, gamma, scale, tol

    def fit(self, X: torch.Tensor, y: torch.Tensor) -> "SVC":
        X = X.double()
        if self.scale:
            self.mu = X.mean(0)
            sd = X.std(0)
            self.sd = torch.where(sd > 0, sd, torch.ones_like(sd))
            X = (X - self.mu) / self.sd
        self.gamma_ = self.gamma if self.gamma is not None else 1.0 / X.shape[1]
        yy = torch.where(y.to(X.device) > 0, 1.0, -1.0).double()
        K = kernel_matrix(X, X, self.kernel, self.gamma_).cpu().numpy()
        a, b = smo(K, yy.cpu().numpy(), self.C, self.tol)
        sv = np.nonzero(a > 1e-12)[0]
        self.support_ = torch.as_tensor(sv, device=X.device)
        self.SV = X[self.support_]
        self.coefs = torch.as_tensor(a[sv] * yy.cpu().numpy()[sv], device=X.device)   # a_i y_i
        self.b = float(b)
        return self

    def _prep(self, X):
        X = X.double()
        return (X - self.mu) / self.sd if self.scale else X

    def decision_function(self, X: torch.Tensor) -> torch.Tensor:
        Kx = kernel_matrix(self._prep(X), self.SV, self.kernel, self.gamma_)
        return Kx @ self.coefs + self.b

    def predict(self, X: torch.Tensor) -> torch.Tensor:
        return (self.decision_function(X) > 0).long()

    @property
    def weights(self) -> Optional[torch.Tensor]:
        """w = t(coefs) %*% SV (scaled space) — only meaningful for the linear kernel."""
        if self.kernel != "linear":
            return None
        return self.coefs @ self.SV


def run_svm(seed: int, kernel: str, X_train: torch.Tensor, y_train: torch.Tensor,
            X_test: torch.Tensor, y_test: torch.Tensor, weightfilt: Optional[float] = None,
            feature_names: Optional[Sequence[str]] = None) -> Dict[str, object]:
    """runSVM: fit, optional top-|w| fraction refit, train/test decisions, ROC, precision,
    recall. Keys follow the reference (snake_case)."""
    torch.manual_seed(seed)
    names = list(feature_names) if feature_names is not None else [str(i) for i in range(X_train.shape[1])]
    opts = []
    m = SVC(kernel).fit(X_train, y_train)
    cols = torch.arange(X_train.shape[1], device=X_train.device)
    if weightfilt:
        w = m.weights
        if w is None:    # radial: rank features by the linear SVM's weights instead
            w = SVC("linear").fit(X_train, y_train).weights
        k = int(round(X_train.shape[1] * weightfilt))
        cols = torch.argsort(w.abs(), descending=True)[:k]
        opts.append(f"weight filt = {weightfilt}")
        opts.append("cols_retained: " + ";".join(names[i] for i in cols.cpu().tolist()))
        m = SVC(kernel).fit(X_train[:, cols], y_train)
    else:
        opts.append("no weight filt")
    dtr = m.decision_function(X_train[:, cols])
    dte = m.decision_function(X_test[:, cols])
    ptr, pte = (dtr > 0).long().cpu(), (dte > 0).long().cpu()
    yt = y_test.long().cpu()
    fpr, tpr, _ = roc_curve(yt, dte.cpu())
    met = binary_metrics(yt, pte)
    w = m.weights
    weights_full = None
    if w is not None:
        weights_full = torch.zeros(X_train.shape[1], dtype=torch.float64, device=w.device)
        weights_full[cols] = w
    return {"options_string": opts, "svm_model": m, "weightsvect": weights_full,
            "features_used": [names[i] for i in cols.cpu().tolist()],
            "predictions_train": ptr, "predictions_test": pte,
            "decision_values_test": dte.cpu(), "performance_test": {"fpr": fpr, "tpr": tpr},
            "TPR_test": met["tpr"], "precision_test": met["precision"],
            "recall_test": met["recall"], "test_metrics": met}


def weight_quantile_genes(weights: torch.Tensor, names: Sequence[str],
                          quantiles=(0.25, 0.10, 0.05, 0.01, 0.001)) -> Dict[str, Dict[float, list]]:
    """Top / bottom weight quantile gene lists (C33, `BuieRProj/KM_WHATEVER.Rmd:315-351`)."""
    w = weights.double().cpu()
    order = torch.argsort(w)
    n = w.numel()
    out = {"high": {}, "low": {}}
    for q in quantiles:
        k = max(1, int(round(q * n)))
        out["low"][q] = [names[i] for i in order[:k].tolist()]
        out["high"][q] = [names[i] for i in order.flip(0)[:k].tolist()]
    return out
