"""C-support-vector classification (C23, C33): libsvm-style SMO on a precomputed kernel matrix,
e1071 semantics (``scale=TRUE`` column standardisation, cost 1, radial gamma = 1/p), the primal
weight vector w = sum_i alpha_i y_i x_i, and ``run_svm`` with the weight-filter refit.

Reference: ``runSVM`` (`composite_code/rnotebook/cml_targetaml_seanalysis.Rmd:126-210`). Its
``weightsvect`` is taken BEFORE the weight-filter refit and is meaningless for the radial kernel
(SURVEY.md §4.3); here the weights always come from the model that is returned, and radial
models report ``weights=None``.

The Gram / kernel matrix (n x n, n ~ 100) is one GEMM on the device; SMO (a few hundred O(n)
steps with libsvm's second-order working-set selection) runs on the device too, one wave64 per
problem (``csrc/kernels/svm_smo.hip``), so independent fits (CV folds x cost grid, the four
runSVM configurations) are solved in ONE launch by ``smo_batched`` / ``fit_svcs``. CPU tensors
use the numpy oracle ``smo`` with the same selection order.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

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


def smo(K: np.ndarray, y: np.ndarray, C: float = 1.0, tol: float = 1e-3, max_iter: int = 100000,
        return_grad: bool = False):
    """Dual C-SVC: min 1/2 a^T Q a - e^T a, 0 <= a <= C, y^T a = 0 (Q = y y^T * K).
    Returns (alpha, b) with the decision function sum_i a_i y_i K(x_i, x) + b. Host oracle of the
    batched GPU solver ``smo_batched`` (csrc/kernels/svm_smo.hip), same selection order."""
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
        # second-order working set selection (libsvm WSS2): a_it = Q_ii + Q_tt - 2 y_i y_t Q_it
        #                                                        = K_ii + K_tt - 2 K_it
        b_ = gmax - v
        a_ = K[i, i] + np.diag(K) - 2 * K[i]
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
    if return_grad:
        return a, G
    return a, _bias(a, G, y, C)


def _bias(a, G, y, C) -> float:
    """-rho of libsvm: mean of y G over free SVs, else the middle of the feasible interval."""
    a, G, y = (np.asarray(v) for v in (a, G, y))
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
    return float(-rho)


def smo_batched(Ks, ys, C=1.0, tol: float = 1e-3, max_iter: int = 100000):
    """Solve several dual C-SVC problems at once: one wave64 per problem on the GPU
    (``svm_smo.hip``), the host oracle per problem on CPU. ``Ks``: list of [n_b, n_b] kernel
    matrices (or one [B, n, n] tensor), ``ys``: labels (> 0 -> +1), ``C``: scalar or per problem.
    Returns a list of (alpha [n_b] fp64 tensor, b float, iterations)."""
    Ks = list(Ks)
    ys = list(ys)
    B = len(Ks)
    Cs = [float(C)] * B if np.isscalar(C) else [float(c) for c in C]
    dev = Ks[0].device if torch.is_tensor(Ks[0]) else torch.device("cpu")
    if dev.type == "cuda":
        from ..ops.native import lib
        ns = [int(k.shape[0]) for k in Ks]
        nmax = max(ns)
        if nmax <= lib().smo_max_n():
            Kb = torch.zeros(B, nmax, nmax, dtype=torch.float64, device=dev)
            Yb = torch.ones(B, nmax, dtype=torch.float64, device=dev)
            for b, (k, yv) in enumerate(zip(Ks, ys)):
                Kb[b, :ns[b], :ns[b]] = k.double()
                Yb[b, :ns[b]] = torch.where(yv.to(dev) > 0, 1.0, -1.0).double()
            Cd = torch.tensor(Cs, dtype=torch.float64, device=dev)
            A, G, it = lib().svm_smo(Kb, Yb, ns, Cd, float(tol), int(max_iter))
            A, G, it, Yh = A.cpu().numpy(), G.cpu().numpy(), it.cpu().tolist(), Yb.cpu().numpy()
            return [(torch.as_tensor(A[b, :ns[b]], device=dev),
                     _bias(A[b, :ns[b]], G[b, :ns[b]], Yh[b, :ns[b]], Cs[b]), it[b])
                    for b in range(B)]
    out = []
    for k, yv, c in zip(Ks, ys, Cs):
        kk = k.double().cpu().numpy() if torch.is_tensor(k) else np.asarray(k, dtype=np.float64)
        yy = np.where(np.asarray(yv.cpu() if torch.is_tensor(yv) else yv) > 0, 1.0, -1.0)
        a, G = smo(kk, yy, c, tol, max_iter, return_grad=True)
        out.append((torch.as_tensor(a, device=dev), _bias(a, G, yy, c), -1))
    return out


class SVC:
    def __init__(self, kernel: str = "linear", C: float = 1.0, gamma: Optional[float] = None,
                 scale: bool = True, tol: float = 1e-3):
        self.kernel, self.C, self.gamma, self.scale, self.tol = kernel, C, gamma, scale, tol

    def _problem(self, X: torch.Tensor, y: torch.Tensor):
        """Scaled training data, +-1 labels and the kernel matrix of one fit."""
        X = X.double()
        if self.scale:
            self.mu = X.mean(0)
            sd = X.std(0)
            self.sd = torch.where(sd > 0, sd, torch.ones_like(sd))
            X = (X - self.mu) / self.sd
        self.gamma_ = self.gamma if self.gamma is not None else 1.0 / X.shape[1]
        yy = torch.where(y.to(X.device) > 0, 1.0, -1.0).double()
        return X, yy, kernel_matrix(X, X, self.kernel, self.gamma_)

    def fit(self, X: torch.Tensor, y: torch.Tensor) -> "SVC":
        X, yy, K = self._problem(X, y)
        ((a, b, self.n_iter_),) = smo_batched([K], [yy], self.C, self.tol)
        return self._set_solution(X, yy, a, b)

    def _set_solution(self, X, yy, a, b) -> "SVC":
        sv = torch.nonzero(a > 1e-12).flatten()
        self.support_ = sv
        self.SV = X[sv]
        self.coefs = (a[sv] * yy[sv]).to(X.device)          # a_i y_i
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


def fit_svcs(Xs: Sequence[torch.Tensor], ys: Sequence[torch.Tensor], kernel: str = "linear",
             C=1.0, gamma=None, scale: bool = True, tol: float = 1e-3) -> List[SVC]:
    """Fit independent SVMs (CV folds, cost grids) with ONE batched SMO launch on the GPU.
    ``C`` and ``gamma``: one value, or one per problem."""
    Cs = [C] * len(Xs) if np.isscalar(C) else list(C)
    gs = list(gamma) if isinstance(gamma, (list, tuple)) else [gamma] * len(Xs)
    models = [SVC(kernel, c, g, scale, tol) for c, g in zip(Cs, gs)]
    probs = [m._problem(X, y) for m, X, y in zip(models, Xs, ys)]
    sols = smo_batched([p[2] for p in probs], [p[1] for p in probs], Cs, tol)
    for m, (X, yy, _), (a, b, it) in zip(models, probs, sols):
        m.n_iter_ = it
        m._set_solution(X, yy, a, b)
    return models


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
