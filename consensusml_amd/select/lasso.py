"""L1-penalised logistic regression along a lambda path with batched cross-validation (C17, C20,
C21, C22).

Reference: ``runLasso`` (`composite_code/rnotebook/cml_targetaml_seanalysis.Rmd:68-123`) fits
glmnet binomial lasso (alpha 1, no intercept, no standardisation, lambda = 10^seq(10, -2, 100)),
picks lambda.min by leave-one-out CV on misclassification (`:98-101`), reports test error, refits
on all samples and returns the nonzero coefficients; ``glm.binom``
(`JSmith_code/Differential_Expression_and_Lasso.Rmd:302-391`) is the same with an intercept;
the 15 iterative-exclusion reps live at `...seanalysis.Rmd:727-778`. The hot loop there is
93 LOOCV folds x 100 lambdas x 15 reps of serial Fortran coordinate descent.

MI355X design: every (fold, lambda) pair is one column of a coefficient matrix B [p, folds*L].
One FISTA iteration for ALL problems is two GEMMs (Z = X B, G = X^T R on hipBLASLt through
torch.matmul) plus elementwise residual / soft-threshold passes, so the whole LOOCV path is a
few hundred batched iterations instead of ~9,300 sequential fits. Objective per problem
(glmnet's): (1/n_b) sum_i m_ib [log(1 + e^{z_i}) - y_i z_i] + lambda_b ||beta||_1, intercept
unpenalised when present. Folds can be sharded over ranks (ensemble parallelism).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from .metrics import binary_metrics, confusion_matrix

GLMNET_GRID = 10.0 ** np.linspace(10, -2, 100)


@dataclass
class LassoPath:
    lambdas: torch.Tensor        # [L]
    coef: torch.Tensor           # [L, p]
    intercept: torch.Tensor      # [L]
    iters: int
    converged: bool

    def at(self, lam: float):
        i = int(torch.argmin((self.lambdas - lam).abs()))
        return self.coef[i], self.intercept[i]


def _soft(x: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    return torch.sign(x) * torch.clamp(x.abs() - t, min=0.0)


def fista_logistic(X: torch.Tensor, y: torch.Tensor, lambdas: torch.Tensor,
                   masks: Optional[torch.Tensor] = None, intercept: bool = False,
                   max_iter: int = 3000, tol: float = 1e-6, check_every: int = 25,
                   alpha: float = 1.0):
    """Solve B independent elastic-net logistic problems at once.

    X [n, p], y [n] in {0, 1}, lambdas [B], masks [n, B] sample weights (1 = in the problem).
    Returns (beta [p, B], b0 [B], iterations, converged).
    """
    X = X.float()
    n, p = X.shape
    dev = X.device
    lam = lambdas.to(dev, torch.float32).view(1, -1)
    Bn = lam.shape[1]
    M = torch.ones(n, Bn, device=dev) if masks is None else masks.to(dev, torch.float32)
    nb = M.sum(0, keepdim=True).clamp_min(1.0)
    yv = y.to(dev, torch.float32).view(n, 1)
    # Lipschitz bound of the smooth part: 0.25 * ||X||_2^2 / n_b (+1 for the intercept column)
    s = torch.linalg.matrix_norm(X, ord=2).item() ** 2
    if intercept:
        s += n
    step = 1.0 / (0.25 * s / nb + lam * (1 - alpha))
    if dev.type == "cuda":
        return _fista_gpu(X, yv.view(-1), lam.view(-1), M, nb.view(-1), step.view(-1), intercept,
                          max_iter, tol, check_every, alpha)
    out_beta = torch.zeros(p, Bn, device=dev)
    out_b0 = torch.zeros(1, Bn, device=dev)
    # working set of unconverged problems; converged columns are written out and dropped, so
    # the batch shrinks as the easy (large-lambda) problems finish
    act = torch.arange(Bn, device=dev)
    beta = out_beta.clone()
    b0 = out_b0.clone()
    v, v0 = beta.clone(), b0.clone()
    tk = torch.ones(1, Bn, device=dev)
    Ma, nba, lama, stepa = M, nb, lam, step
    it = 0
    for it in range(1, max_iter + 1):
        z = X @ v + v0
        r = (torch.sigmoid(z) - yv) * Ma / nba                   # d loss / d z
        g = X.t() @ r
        if alpha < 1:
            g = g + lama * (1 - alpha) * v
        nbeta = _soft(v - stepa * g, stepa * lama * alpha)
        nb0 = v0 - stepa * r.sum(0, keepdim=True) if intercept else b0
        # adaptive restart (O'Donoghue & Candes): drop momentum where it points uphill
        up = ((v - nbeta) * (nbeta - beta)).sum(0, keepdim=True) > 0
        tn = (1 + torch.sqrt(1 + 4 * tk * tk)) / 2
        mom = torch.where(up, torch.zeros_like(tk), (tk - 1) / tn)
        tk = torch.where(up, torch.ones_like(tk), tn)
        d = nbeta - beta
        v = nbeta + mom * d
        v0 = nb0 + mom * (nb0 - b0) if intercept else nb0
        beta, b0 = nbeta, nb0
        if it % check_every == 0 or it == max_iter:
            delta = d.abs().amax(0) / beta.abs().amax(0).clamp_min(1.0)
            done = delta < tol
            if bool(done.any()) or it == max_iter:
                keep = ~done if it < max_iter else torch.zeros_like(done)
                fin = act[~keep]
                out_beta[:, fin] = beta[:, ~keep]
                out_b0[:, fin] = b0[:, ~keep]
                if not bool(keep.any()):
                    break
                act = act[keep]
                beta, b0, v, v0, tk = beta[:, keep], b0[:, keep], v[:, keep], v0[:, keep], tk[:, keep]
                Ma, nba, lama, stepa = Ma[:, keep], nba[:, keep], lama[:, keep], stepa[:, keep]
    converged = it < max_iter
    return out_beta, out_b0.view(-1), it, converged


def _fista_gpu(X, y, lam, M, nb, step, intercept, max_iter, tol, check_every, alpha):
    """fista_logistic on the GPU: the two GEMMs per iteration on hipBLASLt, the residual and the
    prox / adaptive-restart / momentum update as the fused kernels of csrc/kernels/lasso_prox.hip
    (same iteration, same working-set shrinking; no host sync between convergence checks)."""
    from ..ops.native import lib
    C = lib()
    n, p = X.shape
    dev = X.device
    Bn = lam.numel()
    ns = C.lasso_slices(p)
    out_beta = torch.zeros(p, Bn, device=dev)
    out_b0 = torch.zeros(Bn, device=dev)
    act = torch.arange(Bn, device=dev)
    beta = torch.zeros(p, Bn, device=dev)
    v = torch.zeros(p, Bn, device=dev)
    b0 = torch.zeros(Bn, device=dev)
    v0 = torch.zeros(Bn, device=dev)
    tk = torch.ones(Bn, device=dev)
    Ma, nba, lama, stepa = M.contiguous(), nb.contiguous(), lam.contiguous(), step.contiguous()
    Xt = X.t().contiguous()

    def scratch(B):
        return (torch.empty(p, B, device=dev), torch.empty(B, device=dev),
                torch.empty(ns, B, device=dev), torch.empty(ns, 2, B, device=dev),
                torch.empty(n, B, device=dev), torch.empty(B, device=dev))

    nbuf, mom, part, conv, r, rsum = scratch(Bn)
    it = 0
    for it in range(1, max_iter + 1):
        z = X @ v
        C.lasso_resid(z, v0 if intercept else None, y, Ma, nba, r, rsum if intercept else None)
        g = Xt @ r
        check = it % check_every == 0 or it == max_iter
        C.lasso_step(v, beta, g, stepa, lama, float(alpha), tk, rsum if intercept else None,
                     v0 if intercept else None, b0 if intercept else None, nbuf, mom, part,
                     conv if check else None)
        if check:
            delta = conv[:, 0].amax(0) / conv[:, 1].amax(0).clamp_min(1.0)
            done = delta < tol
            if bool(done.any()) or it == max_iter:
                keep = ~done if it < max_iter else torch.zeros_like(done)
                fin = act[~keep]
                out_beta[:, fin] = beta[:, ~keep]
                out_b0[fin] = b0[~keep]
                if not bool(keep.any()):
                    break
                act = act[keep]
                beta, v = beta[:, keep].contiguous(), v[:, keep].contiguous()
                b0, v0, tk = b0[keep].contiguous(), v0[keep].contiguous(), tk[keep].contiguous()
                Ma = Ma[:, keep].contiguous()
                nba, lama, stepa = nba[keep].contiguous(), lama[keep].contiguous(), stepa[keep].contiguous()
                nbuf, mom, part, conv, r, rsum = scratch(int(keep.sum()))
    converged = it < max_iter
    return out_beta, out_b0, it, converged


def lasso_path(X: torch.Tensor, y: torch.Tensor, lambdas: Sequence[float] = GLMNET_GRID,
               intercept: bool = False, **kw) -> LassoPath:
    lam = torch.as_tensor(np.asarray(lambdas, dtype=np.float32), device=X.device)
    beta, b0, it, ok = fista_logistic(X, y, lam, intercept=intercept, **kw)
    return LassoPath(lam, beta.t().contiguous(), b0, it, ok)


def cv_lasso(X: torch.Tensor, y: torch.Tensor, lambdas: Sequence[float] = GLMNET_GRID,
             nfolds: Optional[int] = None, intercept: bool = False, seed: int = 2019,
             measure: str = "class", shard: bool = True, **kw) -> Dict[str, object]:
    """K-fold (default leave-one-out) CV of the whole path; all folds x lambdas in one batch.

    Returns cvm (mean error per lambda), cvsd, lambda_min (largest lambda attaining the minimum,
    glmnet's rule) and lambda_1se.
    """
    n = X.shape[0]
    dev = X.device
    K = n if nfolds is None else nfolds
    g = np.random.default_rng(seed)
    foldid = np.arange(n) if K == n else g.permutation(np.arange(n) % K)
    lam = torch.as_tensor(np.asarray(lambdas, dtype=np.float32), device=dev)
    L = lam.numel()
    folds = list(range(K))
    rank, world = 0, 1
    if shard and dist.is_available() and dist.is_initialized():
        rank, world = dist.get_rank(), dist.get_world_size()
        folds = folds[rank::world]
    err = torch.zeros(K, L, dtype=torch.float64, device=dev)
    cnt = torch.zeros(K, dtype=torch.float64, device=dev)
    fid = torch.as_tensor(foldid, device=dev)
    if folds:
        F = len(folds)
        train_mask = torch.stack([(fid != k).float() for k in folds], 1)     # [n, F]
        masks = train_mask.repeat_interleave(L, 1)                            # [n, F*L]
        lams = lam.repeat(F)
        beta, b0, _, _ = fista_logistic(X, y, lams, masks, intercept, **kw)
        z = X.float() @ beta + b0.view(1, -1)                                 # [n, F*L]
        pred = (z > 0).float()
        yv = y.to(dev).float().view(n, 1)
        if measure == "class":
            e = (pred != yv).double()
        else:   # deviance
            pz = torch.sigmoid(z).clamp(1e-6, 1 - 1e-6)
            e = -(yv * pz.log() + (1 - yv) * (1 - pz).log()).double() * 2
        test = (1 - masks).double()
        per = (e * test).sum(0).view(F, L)
        for j, k in enumerate(folds):
            err[k] = per[j]
            cnt[k] = (fid == k).sum()
    if world > 1:
        dist.all_reduce(err)
        dist.all_reduce(cnt)
    fold_err = err / cnt.view(-1, 1).clamp_min(1)                             # [K, L]
    w = cnt / cnt.sum()
    cvm = (fold_err * w.view(-1, 1)).sum(0)
    cvsd = torch.sqrt(((fold_err - cvm) ** 2 * w.view(-1, 1)).sum(0) / max(K - 1, 1))
    lam_np = lam.double().cpu().numpy()
    cvm_np = cvm.cpu().numpy()
    mn = cvm_np.min()
    idmin = np.where(cvm_np <= mn + 1e-12)[0]
    lmin = float(lam_np[idmin].max())
    imin = int(np.where(lam_np == lmin)[0][0])
    l1se = float(lam_np[cvm_np <= mn + cvsd.cpu().numpy()[imin]].max())
    return {"lambda": lam_np, "cvm": cvm_np, "cvsd": cvsd.cpu().numpy(), "lambda_min": lmin,
            "lambda_1se": l1se, "nfolds": K, "foldid": foldid}


def predict_class(path: LassoPath, X: torch.Tensor, lam: float) -> torch.Tensor:
    b, b0 = path.at(lam)
    return ((X.float() @ b + b0) > 0).long()


def polish_cd(X: torch.Tensor, y: torch.Tensor, lam: float, beta: torch.Tensor,
              b0: float = 0.0, intercept: bool = False, tol: float = 1e-13,
              max_outer: int = 100) -> tuple:
    """Exact optimum of ONE lasso-logistic problem, from a warm start: fp64 IRLS outer loop with
    active-set coordinate descent inside (glmnet's algorithm, driven to a tight tolerance), on
    the host. FISTA (the batched path solver) reaches the lambda-path's selection quickly but
    stops at a relative step of 1e-6, a few percent off per coefficient; the final refit the
    reference reports (``coef(final.model, s = lambda.min)``, `...seanalysis.Rmd:110-115`) is
    polished here so the coefficients are the optimum's, not the stopping rule's."""
    Xn = X.double().cpu().numpy()
    yv = y.double().cpu().numpy()
    b = beta.double().cpu().numpy().copy()
    n, p = Xn.shape
    c = float(b0)
    for _ in range(max_outer):
        eta = Xn @ b + c
        pr = 1.0 / (1.0 + np.exp(-eta))
        w = np.clip(pr * (1 - pr), 1e-5, None)
        r = (yv - pr) / w                     # working residual z - eta
        xw2 = (w[:, None] * Xn * Xn).sum(0) / n
        sw = w.sum() / n
        active = np.nonzero(b)[0].tolist()
        for _full in range(50):
            for _sweep in range(10000):       # coordinate descent on the active set
                maxd = 0.0
                for j in active:
                    bj = b[j]
                    g = float((w * Xn[:, j] * r).sum()) / n + xw2[j] * bj
                    nb = math.copysign(max(abs(g) - lam, 0.0), g) / xw2[j]
                    if nb != bj:
                        r -= Xn[:, j] * (nb - bj)
                        b[j] = nb
                        maxd = max(maxd, xw2[j] * (nb - bj) ** 2)
                if intercept:
                    d = float((w * r).sum()) / n / sw
                    r -= d
                    c += d
                    maxd = max(maxd, sw * d * d)
                if maxd < tol:
                    break
            # KKT over every coordinate: admit the violators, else this outer step is done
            g_all = (Xn * (w * r)[:, None]).sum(0) / n
            viol = [j for j in np.nonzero(np.abs(g_all) > lam * (1 + 1e-9))[0].tolist()
                    if b[j] == 0.0]
            if not viol:
                break
            active = sorted(set(active) | set(viol))
        if np.abs(Xn @ b + c - eta).max() < 1e-11:
            break
    return torch.as_tensor(b, dtype=torch.float64), c


def run_lasso(X: torch.Tensor, y: torch.Tensor, genes: Sequence[str], train_idx: Sequence[int],
              test_idx: Sequence[int], seed: int = 2019, intercept: bool = False,
              lambdas: Sequence[float] = GLMNET_GRID, levels=("0", "1"), polish: bool = True,
              **kw) -> Dict[str, object]:
    """runLasso / glm.binom: returns the reference's named result list (snake_case keys).
    ``polish``: the reported final coefficients are the exact optimum at lambda.min
    (``polish_cd``) rather than the batched path solver's stopping point."""
    torch.manual_seed(seed)
    dev = X.device
    tr = torch.as_tensor(list(train_idx), device=dev)
    te = torch.as_tensor(list(test_idx), device=dev)
    Xtr, ytr = X[tr], y[tr]
    fit = lasso_path(Xtr, ytr, lambdas, intercept, **kw)
    cv = cv_lasso(Xtr, ytr, lambdas, None, intercept, seed, **kw)
    pred = predict_class(fit, X[te], cv["lambda_min"]).cpu()
    yt = y[te].long().cpu()
    tab = confusion_matrix(yt, pred, 2)
    final = lasso_path(X, y, lambdas, intercept, **kw)
    coef, b0 = final.at(cv["lambda_min"])
    if polish:
        pc, pb0 = polish_cd(X, y, float(cv["lambda_min"]), coef, float(b0), intercept)
        coef = pc.to(coef.device, coef.dtype)
        b0 = torch.as_tensor(pb0, dtype=coef.dtype)
    nz = torch.nonzero(coef).flatten().cpu().tolist()
    nonzero = {genes[i]: float(coef[i]) for i in nz}
    if intercept:
        nonzero = {"(Intercept)": float(b0), **nonzero}
    return {"training_set": list(train_idx), "testing_set": list(test_idx),
            "contrast": {levels[0]: 0, levels[1]: 1}, "train_fit": fit, "cv_fit": cv,
            "confusion_matrix": tab, "test_error": float((pred != yt).float().mean()),
            "final_model": final, "nonzero_coef": nonzero, "seed": seed,
            "test_metrics": binary_metrics(yt, pred)}


def iterative_exclusion(X: torch.Tensor, y: torch.Tensor, genes: Sequence[str],
                        train_idx, test_idx, reps: int = 15, seed: int = 2019,
                        **kw) -> List[Dict[str, object]]:
    """Reps of run_lasso, each excluding every gene selected by an earlier rep (C22) — a probe
    of how redundant the predictive signal is. Each result gets ``excluded`` and metrics."""
    excluded: set = set()
    out = []
    for r in range(reps):
        keep = [i for i, g in enumerate(genes) if g not in excluded]
        if not keep:
            break
        kidx = torch.as_tensor(keep, device=X.device)
        res = run_lasso(X[:, kidx], y, [genes[i] for i in keep], train_idx, test_idx, seed, **kw)
        res["rep"] = r + 1
        res["excluded_before"] = sorted(excluded)
        out.append(res)
        excluded |= {g for g in res["nonzero_coef"] if g != "(Intercept)"}
    return out


def l1_logistic_sklearn_like(X: torch.Tensor, y: torch.Tensor, C: float = 1.0,
                             fit_intercept: bool = True, **kw):
    """sklearn ``LogisticRegression(penalty='l1', C)`` objective (C17, `model_walkthrough.ipynb`
    cell 35): ||b||_1 + C sum loss  <=>  lambda = 1 / (C n). Returns (coef [p], intercept)."""
    n = X.shape[0]
    lam = torch.tensor([1.0 / (C * n)], device=X.device)
    beta, b0, _, _ = fista_logistic(X, y, lam, intercept=fit_intercept, **kw)
    return beta[:, 0], float(b0[0])
