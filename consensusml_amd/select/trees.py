"""Tree ensembles with feature importances (C15, C16, C24, C25): gradient boosting
(XGBoost-style second-order, `scripts/model_comp.py:6-34`, `cml_targetaml_seanalysis.Rmd:1148-1239`)
and random forests (Gini, bootstrap, proximity — `...seanalysis.Rmd:1022-1069`).

Split search is vectorised over ALL candidate features of a node at once: the node's rows are
sorted per feature ([m, F] torch.sort), prefix sums of gradient / hessian (or class counts) give
every threshold's gain in one tensor, and the best (threshold, feature) is an argmax. Trees are
stored as flat arrays and predicted level by level. Works on CPU and GPU tensors.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .metrics import log_loss


@dataclass
class Tree:
    feature: List[int] = field(default_factory=list)      # -1 for leaves
    threshold: List[float] = field(default_factory=list)
    left: List[int] = field(default_factory=list)
    right: List[int] = field(default_factory=list)
    value: List[float] = field(default_factory=list)
    leaf_id: List[int] = field(default_factory=list)

    def add(self, feat=-1, thr=0.0, val=0.0) -> int:
        self.feature.append(feat)
        self.threshold.append(thr)
        self.left.append(-1)
        self.right.append(-1)
        self.value.append(val)
        return len(self.feature) - 1

    def predict(self, X: torch.Tensor) -> torch.Tensor:
        return self._route(X, values=True)

    def apply(self, X: torch.Tensor) -> torch.Tensor:
        """Leaf index per row (for forest proximity)."""
        return self._route(X, values=False)

    def _route(self, X: torch.Tensor, values: bool) -> torch.Tensor:
        dev = X.device
        f = torch.tensor(self.feature, device=dev)
        t = torch.tensor(self.threshold, device=dev, dtype=X.dtype)
        l = torch.tensor(self.left, device=dev)
        r = torch.tensor(self.right, device=dev)
        node = torch.zeros(X.shape[0], dtype=torch.long, device=dev)
        for _ in range(64):
            ff = f[node]
            leaf = ff < 0
            if bool(leaf.all()):
                break
            xv = X[torch.arange(X.shape[0], device=dev), ff.clamp_min(0)]
            nxt = torch.where(xv <= t[node], l[node], r[node])
            node = torch.where(leaf, node, nxt)
        if values:
            return torch.tensor(self.value, device=dev, dtype=torch.float32)[node]
        return node


def _best_split(Xn: torch.Tensor, g: torch.Tensor, h: torch.Tensor, crit: str, lam: float,
                min_child: float, min_leaf: int):
    """Best split of one node over the given feature columns.

    crit 'xgb': gain = G_L^2/(H_L+lam) + G_R^2/(H_R+lam) - G^2/(H+lam) (halved like XGBoost)
    crit 'gini': weighted Gini decrease with g = 1{y=1}, h = 1.
    Returns (gain, feature_col, threshold) or None.
    """
    m, F = Xn.shape
    if m < 2 * max(min_leaf, 1):
        return None
    vals, order = torch.sort(Xn, dim=0, stable=True)
    if crit == "xgb":
        # XGBoost's exact greedy split arithmetic: float gradient pairs summed in double, the
        # split's loss change formed in double and stored as a float (SplitEntry::loss_chg), a
        # split only when that float exceeds kRtEps = 1e-6, ties to the lower feature index and,
        # within a feature, to the first threshold of the ascending scan (SplitEntry::NeedReplace).
        # Float sums and a flat argmax split near-tied deep-tree nodes differently
        # (tests/test_reference_rdata_parity.py::test_xgb_importance_parity).
        G = torch.cumsum(g[order].double(), 0)
        H = torch.cumsum(h[order].double(), 0)
        Gt, Ht = G[-1:], H[-1:]
        GL, HL = G[:-1], H[:-1]
        GR, HR = Gt - GL, Ht - HL
        chg = (GL * GL / (HL + lam) + GR * GR / (HR + lam) - Gt * Gt / (Ht + lam)).float()
        ok = (HL >= min_child) & (HR >= min_child) & (vals[1:] > vals[:-1])
        chg = torch.where(ok, chg, torch.full_like(chg, -float("inf")))
        kbest = torch.argmax(chg, dim=0)                       # first max per feature
        fbest = chg.gather(0, kbest.view(1, -1)).view(-1)
        j = int(torch.argmax(fbest))                           # first (lowest) feature of the max
        k = int(kbest[j])
        best = float(fbest[j])
        if not math.isfinite(best) or best <= 1e-6:
            return None
        thr = float((vals[k, j] + vals[k + 1, j]) / 2)
        return 0.5 * best, j, thr
    G = torch.cumsum(g[order], 0)
    H = torch.cumsum(h[order], 0)
    Gt, Ht = G[-1:], H[-1:]
    GL, HL = G[:-1], H[:-1]
    GR, HR = Gt - GL, Ht - HL
    if False:
        pass
    else:
        def gini_w(pos, n):   # n * gini impurity
            p = pos / n.clamp_min(1e-12)
            return n * (1 - p * p - (1 - p) * (1 - p))
        gain = gini_w(Gt, Ht) - gini_w(GL, HL) - gini_w(GR, HR)
        ok = (HL >= min_leaf) & (HR >= min_leaf)
    ok = ok & (vals[1:] > vals[:-1])
    gain = torch.where(ok, gain, torch.full_like(gain, -float("inf")))
    flat = int(torch.argmax(gain))
    k, j = divmod(flat, F)
    best = float(gain[k, j])
    if not math.isfinite(best) or best <= 1e-12:
        return None
    thr = float((vals[k, j] + vals[k + 1, j]) / 2)
    return best, j, thr


def grow_tree(X: torch.Tensor, g: torch.Tensor, h: torch.Tensor, rows: torch.Tensor,
              max_depth: int, crit: str, lam: float = 1.0, min_child: float = 1.0,
              min_leaf: int = 1, feat_frac: float = 1.0, feat_per_node: Optional[int] = None,
              gen: Optional[torch.Generator] = None, importance: Optional[torch.Tensor] = None,
              leaf_value=None, tree_feats: Optional[torch.Tensor] = None) -> Tree:
    """Depth-first growth; ``leaf_value(g_rows, h_rows)`` gives the leaf output."""
    p = X.shape[1]
    tree = Tree()
    all_feats = tree_feats if tree_feats is not None else torch.arange(p, device=X.device)

    def build(idx: torch.Tensor, depth: int) -> int:
        gi, hi = g[idx], h[idx]
        node = tree.add(val=float(leaf_value(gi, hi)))
        if depth >= max_depth or idx.numel() < 2:
            return node
        feats = all_feats
        if feat_per_node is not None and feat_per_node < feats.numel():
            pick = torch.randperm(feats.numel(), generator=gen, device="cpu")[:feat_per_node]
            feats = feats[pick.to(feats.device)]
        res = _best_split(X[idx][:, feats], gi, hi, crit, lam, min_child, min_leaf)
        if res is None:
            return node
        gain, j, thr = res
        f = int(feats[j])
        go_left = X[idx, f] <= thr
        li, ri = idx[go_left], idx[~go_left]
        if li.numel() == 0 or ri.numel() == 0:
            return node
        tree.feature[node] = f
        tree.threshold[node] = thr
        if importance is not None:
            importance[f] += gain
        tree.left[node] = build(li, depth + 1)
        tree.right[node] = build(ri, depth + 1)
        return node

    build(rows, 0)
    return tree


# ============================================================================ gradient boosting
class GradientBoostedTrees:
    """Binary-logistic boosting. ``style='xgb'`` = XGBoost defaults of the reference
    (lr, depth, lambda 1, min_child_weight 1, gain importance); ``style='sklearn'`` adds
    row subsampling / log2 feature sampling like sklearn's GradientBoostingClassifier as used at
    `scripts/model_comp.py:8`."""

    def __init__(self, n_estimators: int = 100, learning_rate: float = 0.3, max_depth: int = 6,
                 reg_lambda: float = 1.0, min_child_weight: float = 1.0, subsample: float = 1.0,
                 colsample: float = 1.0, max_features: Optional[str] = None, seed: int = 8):
        self.n = n_estimators
        self.lr = learning_rate
        self.depth = max_depth
        self.lam = reg_lambda
        self.mcw = min_child_weight
        self.subsample = subsample
        self.colsample = colsample
        self.max_features = max_features
        self.seed = seed
        self.trees: List[Tree] = []
        self.base = 0.0

    def fit(self, X: torch.Tensor, y: torch.Tensor) -> "GradientBoostedTrees":
        X = X.float()
        y = y.float().to(X.device)
        n, p = X.shape
        gen = torch.Generator().manual_seed(self.seed)
        self.base = 0.0                       # XGBoost base_score 0.5 -> margin 0
        margin = torch.zeros(n, device=X.device)
        self.importance = torch.zeros(p, dtype=torch.float64)
        imp = torch.zeros(p, dtype=torch.float64)
        self.trees = []
        fpn = None
        if self.max_features == "log2":
            fpn = max(1, int(math.log2(p)))
        elif self.max_features == "sqrt":
            fpn = max(1, int(math.sqrt(p)))
        for _ in range(self.n):
            pr = torch.sigmoid(margin)
            g = pr - y
            h = (pr * (1 - pr)).clamp_min(1e-16)
            rows = torch.arange(n, device=X.device)
            if self.subsample < 1:
                k = max(2, int(round(self.subsample * n)))
                rows = rows[torch.randperm(n, generator=gen)[:k].to(X.device)]
            tf = None
            if self.colsample < 1:
                k = max(1, int(round(self.colsample * p)))
                tf = torch.randperm(p, generator=gen)[:k].to(X.device)
            lam = self.lam
            t = grow_tree(X, g, h, rows, self.depth, "xgb", lam, self.mcw, 1, 1.0, fpn, gen,
                          imp, leaf_value=lambda gg, hh: -gg.sum() / (hh.sum() + lam),
                          tree_feats=tf)
            self.trees.append(t)
            margin = margin + self.lr * t.predict(X)
        self.importance = imp
        return self

    def decision_function(self, X: torch.Tensor) -> torch.Tensor:
        X = X.float()
        m = torch.full((X.shape[0],), self.base, device=X.device)
        for t in self.trees:
            m = m + self.lr * t.predict(X)
        return m

    def predict_proba(self, X: torch.Tensor) -> torch.Tensor:
        p1 = torch.sigmoid(self.decision_function(X))
        return torch.stack([1 - p1, p1], 1)

    @property
    def feature_importances_(self) -> torch.Tensor:
        s = self.importance.sum()
        return self.importance / s if s > 0 else self.importance


# ============================================================================ random forest
class RandomForest:
    """CART classification forest (Gini), bootstrap rows, sqrt(p) features per node;
    ``mean_decrease_gini`` is R randomForest's importance; ``proximity`` the N x N matrix."""

    def __init__(self, n_estimators: int = 500, max_depth: Optional[int] = None,
                 max_features: str = "sqrt", min_samples_leaf: int = 1, seed: int = 8):
        self.n = n_estimators
        self.depth = max_depth if max_depth is not None else 64
        self.max_features = max_features
        self.min_leaf = min_samples_leaf
        self.seed = seed
        self.trees: List[Tree] = []

    def fit(self, X: torch.Tensor, y: torch.Tensor) -> "RandomForest":
        X = X.float()
        yv = y.float().to(X.device)
        n, p = X.shape
        gen = torch.Generator().manual_seed(self.seed)
        fpn = max(1, int(math.sqrt(p))) if self.max_features == "sqrt" else (
            max(1, int(math.log2(p))) if self.max_features == "log2" else p)
        imp = torch.zeros(p, dtype=torch.float64)
        ones = torch.ones(n, device=X.device)
        self.trees = []
        for _ in range(self.n):
            rows = torch.randint(0, n, (n,), generator=gen).to(X.device)
            t = grow_tree(X, yv, ones, rows, self.depth, "gini", min_leaf=self.min_leaf,
                          feat_per_node=fpn, gen=gen, importance=imp,
                          leaf_value=lambda gg, hh: gg.sum() / hh.sum())
            self.trees.append(t)
        self.mean_decrease_gini = imp / self.n / max(n, 1) * n   # summed decrease / ntree
        self.importance = imp
        return self

    def predict_proba(self, X: torch.Tensor) -> torch.Tensor:
        X = X.float()
        p1 = torch.stack([t.predict(X) for t in self.trees]).mean(0)
        return torch.stack([1 - p1, p1], 1)

    def predict(self, X: torch.Tensor) -> torch.Tensor:
        return (self.predict_proba(X)[:, 1] > 0.5).long()

    def proximity(self, X: torch.Tensor) -> torch.Tensor:
        leaves = torch.stack([t.apply(X.float()) for t in self.trees])       # [T, N]
        same = (leaves[:, :, None] == leaves[:, None, :]).float().mean(0)
        return same

    @property
    def feature_importances_(self) -> torch.Tensor:
        s = self.importance.sum()
        return self.importance / s if s > 0 else self.importance


# ============================================================================ reference API
def tree_ensemble_compare(X_train, X_test, y_train, y_test, seed: int = 8) -> Dict[str, object]:
    """``model_comp`` (C15): XGB (lr .01, depth 3, 700 trees), GB (lr .01, depth 4, log2 features,
    280 trees, subsample .25) and RF (300 trees, depth 3); probability-averaged ensemble and
    the four test log-losses. Returns all three models (the reference dropped GB, §4.3)."""
    xgb = GradientBoostedTrees(700, 0.01, 3, seed=seed).fit(X_train, y_train)
    gb = GradientBoostedTrees(280, 0.01, 4, reg_lambda=0.0, min_child_weight=0.0,
                              subsample=0.25, max_features="log2", seed=seed).fit(X_train, y_train)
    rf = RandomForest(300, 3, seed=seed).fit(X_train, y_train)
    p = {k: m.predict_proba(X_test)[:, 1].cpu() for k, m in
         (("xgb", xgb), ("gb", gb), ("rf", rf))}
    ens = (p["xgb"] + p["gb"] + p["rf"]) / 3
    yt = y_test.cpu()
    return {"xgb": xgb, "gb": gb, "rf": rf,
            "log_loss": {"ensemble": log_loss(yt, ens), "gb": log_loss(yt, p["gb"]),
                         "rf": log_loss(yt, p["rf"]), "xgb": log_loss(yt, p["xgb"])},
            "ensemble_proba": ens}


def xgboost_tuner(X_train, X_test, y_train, y_test, n_estimators_num: Sequence[int],
                  seed: int = 8) -> Dict[int, float]:
    """C16: test log-loss for 100*k trees, k in n_estimators_num (lr 0.01)."""
    out = {}
    for k in n_estimators_num:
        m = GradientBoostedTrees(100 * k, 0.01, 6, seed=seed).fit(X_train, y_train)
        out[100 * k] = log_loss(y_test.cpu(), m.predict_proba(X_test)[:, 1].cpu())
    return out


# ============================================================================ R result lists
def _perf_testset(y_test: torch.Tensor, prob1: torch.Tensor) -> Dict[str, object]:
    """``performance_testset`` of the XGB result list (`cml_targetaml_seanalysis.Rmd:1198-1224`):
    confusion matrix (rows predicted 0/1, cols observed 0/1), mean_err, tpr, tnr, fdr, for —
    computed from THIS model's predictions (the reference reused a stale ``pred1``, §4.3)."""
    yt = y_test.cpu().long()
    pb = (prob1.cpu() > 0.5).long()
    cm = torch.zeros(2, 2, dtype=torch.long)
    for a, b in zip(pb.tolist(), yt.tolist()):
        cm[a, b] += 1
    tp, fp, tn, fn = int(cm[1, 1]), int(cm[1, 0]), int(cm[0, 0]), int(cm[0, 1])
    pos, neg = int((yt == 1).sum()), int((yt == 0).sum())

    def div(a, b):
        return a / b if b else float("nan")
    return {"confusion_matrix": cm, "mean_err": float((pb != yt).float().mean()),
            "tpr": div(tp, pos), "tnr": div(tn, neg), "fdr": 1 - div(tp, tp + fp),
            "for": 1 - div(tn, tn + fn)}


XGB_REPS = ((2, 1.0, 2), (50, 1.0, 2), (50, 1.0, 50), (100, 1.0, 50), (100, 1.0, 100))


def xgb_resultslist(X_train, y_train, X_test, y_test, reps=XGB_REPS, seed: int = 8):
    """C25 (`cml_targetaml_seanalysis.Rmd:1148-1239`): the five xgboost configs
    (max_depth, eta, nrounds); per rep ``{"model", "importance", "performance_testset"}`` plus
    ``"testperfdf"`` (pandas, rows rep1..repK, cols mean_err/tpr/tnr/fdr/for)."""
    import pandas as pd
    out: Dict[str, object] = {}
    rows = []
    for i, (depth, eta, rounds) in enumerate(reps, 1):
        m = GradientBoostedTrees(rounds, eta, depth, seed=seed).fit(X_train, y_train)
        perf = _perf_testset(y_test, m.predict_proba(X_test)[:, 1])
        out[f"rep{i}"] = {"model": m, "importance": m.feature_importances_,
                          "performance_testset": perf, "params": {"max_depth": depth, "eta": eta,
                                                                  "nrounds": rounds}}
        rows.append({k: perf[k] for k in ("mean_err", "tpr", "tnr", "fdr", "for")})
    out["testperfdf"] = pd.DataFrame(rows, index=[f"rep{i}" for i in range(1, len(reps) + 1)])
    return out


def rf_resultslist(X_train, y_train, X_test, y_test, ntrees=(2000, 5000, 10000),
                   seed: int = 50, proximity: bool = True):
    """C24 (`cml_targetaml_seanalysis.Rmd:1022-1069`): randomForest with 2k / 5k / 10k trees and
    proximity; ``{"rf2k_results": {"fitmodel", "conf_matrix", "proximity",
    "mean_decrease_gini"}, ...}`` with conf_matrix rows observed / cols predicted like R's
    ``table(observed, predicted)``. Trees are grown with the device histogram forest."""
    from .hist_trees import HistForest
    out: Dict[str, object] = {}
    yt = y_test.cpu().long()
    for T in ntrees:
        m = HistForest(T, max_depth=12, seed=seed).fit(X_train, y_train)
        pred = m.predict(X_test).cpu()
        cm = torch.zeros(2, 2, dtype=torch.long)
        for a, b in zip(yt.tolist(), pred.tolist()):
            cm[a, b] += 1
        key = f"rf{T // 1000}k_results" if T % 1000 == 0 else f"rf{T}_results"
        out[key] = {"fitmodel": m, "conf_matrix": cm, "mean_decrease_gini": m.mean_decrease_gini}
        if proximity:
            out[key]["proximity"] = m.proximity(X_train).cpu()
    return out
