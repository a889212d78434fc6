"""Level-synchronous histogram trees: whole forests (and each boosting round) grown as a few
batched device ops per depth level instead of a Python recursion per node.

Features are quantile-binned once (<= 256 bins, uint8). At each depth level every active
(tree, node) pair draws its candidate features, one scatter-add builds all their
(feature, bin) histograms of the split statistics, a cumulative sum over bins scores every
threshold, and an argmax picks each node's split; samples are then routed to children in one
gather. ``HistForest`` (Gini, bootstrap, sqrt(p) features per node, MeanDecreaseGini) and
``HistBoost`` (second-order logistic boosting, XGBoost ``hist`` style) share the grower.

The reference's hot loops — ``randomForest`` with 2k/5k/10k trees (`cml_targetaml_seanalysis.Rmd:
1037-1050`), sklearn RF / GB and XGBoost 700 trees (`scripts/model_comp.py:6-34`) — become
O(depth) launches per chunk of trees.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch


def quantile_bins(X: torch.Tensor, n_bins: int = 64):
    """Per-feature bin edges from the data (midpoints between distinct quantile values).
    Returns (Xb uint8 [n, p], edges float [p, n_bins - 1]) with x <= edges[f, b] <=> bin <= b."""
    X = X.float()
    n, p = X.shape
    qs = torch.linspace(0, 1, n_bins + 1, device=X.device)[1:-1]
    S, _ = torch.sort(X, 0)
    idx = (qs * (n - 1)).round().long()
    lo = S[idx]                                   # [n_bins-1, p]
    hi = S[(idx + 1).clamp_max(n - 1)]
    edges = ((lo + hi) / 2).t().contiguous()      # [p, n_bins-1]
    return bin_with(X, edges), edges


def bin_with(X: torch.Tensor, edges: torch.Tensor) -> torch.Tensor:
    """bin = number of edges strictly below x (one searchsorted over the sorted edge rows)."""
    Xt = X.float().t().contiguous()                                  # [p, n]
    return torch.searchsorted(edges, Xt, right=False).to(torch.uint8).t().contiguous()


def exact_bins(X: torch.Tensor, max_bins: int = 128):
    """Rank bins: every distinct value of a feature gets its own bin, edges at the midpoints
    between consecutive distinct values (R randomForest's candidate thresholds), padded with
    +inf. Returns (Xb uint8 [n, p], edges [p, max_bins - 1], B = most distinct values of any
    feature), or None when some feature has more than ``max_bins`` distinct values."""
    X = X.float()
    S, _ = torch.sort(X, 0)
    mids = (S[1:] + S[:-1]) / 2
    valid = S[1:] > S[:-1]                                   # [n - 1, p]
    B = int(valid.sum(0).max().item()) + 1 if X.shape[0] > 1 else 1
    if B > max_bins:
        return None
    keys = torch.where(valid, mids, torch.full_like(mids, float("inf")))
    keys, _ = torch.sort(keys, 0)                             # valid midpoints first, ascending
    edges = torch.full((X.shape[1], max_bins - 1), float("inf"), device=X.device)
    k = min(max_bins - 1, keys.shape[0])
    edges[:, :k] = keys[:k].t()
    return bin_with(X, edges), edges, max(B, 2)


@dataclass
class TreeBatch:
    feature: torch.Tensor     # [T, nodes] int64, -1 = leaf
    thr_bin: torch.Tensor     # [T, nodes] int64, go left if bin <= thr_bin
    value: torch.Tensor       # [T, nodes] float leaf value
    depth: int

    def predict(self, Xb: torch.Tensor) -> torch.Tensor:
        """Leaf values [T, m] for binned rows Xb [m, p]."""
        return torch.gather(self.value, 1, self.apply(Xb))

    def apply(self, Xb: torch.Tensor) -> torch.Tensor:
        """Leaf node ids [T, m] for binned rows Xb [m, p]."""
        T = self.feature.shape[0]
        m = Xb.shape[0]
        node = torch.zeros(T, m, dtype=torch.long, device=Xb.device)
        ar = torch.arange(m, device=Xb.device)
        for _ in range(self.depth):
            f = torch.gather(self.feature, 1, node).long()
            leaf = f < 0
            b = Xb[ar[None].expand(T, m), f.clamp_min(0)].long()
            thr = torch.gather(self.thr_bin, 1, node).long()
            child = 2 * node + 1 + (b > thr).long()
            node = torch.where(leaf, node, child)
        return node


def grow(Xb: torch.Tensor, stat: torch.Tensor, depth: int, k: int, n_bins: int, crit: str,
         lam: float = 1.0, min_child: float = 1.0, gen: Optional[torch.Generator] = None,
         importance: Optional[torch.Tensor] = None, feat_mask: Optional[torch.Tensor] = None
         ) -> TreeBatch:
    """Grow T trees level by level.

    stat [T, n, 2]: per tree and sample, (w, w*y) for crit 'gini' (w = bootstrap count) or
    (g, h) for crit 'xgb'. k candidate features per node (k = p: all). feat_mask [T, p] bool
    restricts each tree's features (column subsampling).
    """
    dev = Xb.device
    T, n, _ = stat.shape
    p = Xb.shape[1]
    nodes = 2 ** (depth + 1) - 1
    feature = torch.full((T, nodes), -1, dtype=torch.long, device=dev)
    thr = torch.zeros(T, nodes, dtype=torch.long, device=dev)
    value = torch.zeros(T, nodes, device=dev)
    node_of = torch.zeros(T, n, dtype=torch.long, device=dev)   # absolute node id
    alive = stat[..., 0] != 0 if crit == "gini" else torch.ones(T, n, dtype=torch.bool, device=dev)
    tt = torch.arange(T, device=dev)

    def leaf_val(s0, s1):
        if crit == "gini":
            return s1 / s0.clamp_min(1e-12)
        return -s0 / (s1 + lam)

    for level in range(depth + 1):
        L = 2 ** level
        base = L - 1
        local = (node_of - base).clamp(0, L - 1)
        # node totals and leaf values for every node at this level
        key = (tt[:, None] * L + local).view(-1)
        tot = torch.zeros(T * L, 2, device=dev)
        m = alive.view(-1)
        tot.index_add_(0, key[m], stat.view(-1, 2)[m].float())
        tot = tot.view(T, L, 2)
        value[:, base:base + L] = leaf_val(tot[..., 0], tot[..., 1])
        if level == depth:
            break
        # candidate features per (tree, node)
        if k >= p and feat_mask is None:
            feats = torch.arange(p, device=dev).expand(T, L, p)
            kk = p
        else:
            if dev.type == "cuda":
                # candidate draws on the device (a host draw of T x L x p keys, 22M at p = 21k,
                # used to dominate the fit); the device stream is seeded from the host generator
                dgen = torch.Generator(device=dev)
                dgen.manual_seed(int(torch.randint(0, 2 ** 62, (1,), generator=gen)))
                r = torch.rand(T, L, p, generator=dgen, device=dev)
            else:
                r = torch.rand(T, L, p, generator=gen, device="cpu").to(dev)
            if feat_mask is not None:
                r = torch.where(feat_mask[:, None, :], r, torch.full_like(r, -1.0))
            kk = min(k, p) if feat_mask is None else min(k, int(feat_mask.sum(1).min()))
            feats = r.topk(kk, dim=2).indices                     # [T, L, kk]
        if dev.type == "cuda" and n_bins <= 64:
            # csrc/kernels/tree_hist.hip: per-(tree, node) LDS histograms, in-order sums,
            # threshold scan and argmax in one launch
            from ..ops.native import lib
            nl = torch.where(alive, node_of - base, torch.full_like(node_of, -1)).int()
            gbest, jb, bbest = lib().split_search(
                Xb.contiguous(), nl.contiguous(), stat.float().contiguous(), feats.int().contiguous(),
                tot.contiguous(), n_bins, 0 if crit == "gini" else 1, float(lam), float(min_child))
            best, j, b = gbest, jb.long(), bbest.long()
        else:
            best, j, b = _split_search_torch(Xb, stat, feats, local, alive, tot, tt, L, kk,
                                             n_bins, crit, lam, min_child)
        split = torch.isfinite(best) & (best > 1e-12)
        fbest = torch.gather(feats, 2, j[..., None]).squeeze(2)
        feature[:, base:base + L] = torch.where(split, fbest, torch.full_like(fbest, -1))
        thr[:, base:base + L] = b
        if importance is not None:
            gsum = torch.where(split, best, torch.zeros_like(best))
            importance.index_add_(0, fbest.view(-1), gsum.view(-1).double().cpu()
                                  if importance.device.type == "cpu" else gsum.view(-1).double())
        # route samples
        nf = torch.gather(feature[:, base:base + L], 1, local)
        nb = torch.gather(thr[:, base:base + L], 1, local)
        xb = Xb[torch.arange(n, device=dev)[None].expand(T, n), nf.clamp_min(0)].long()
        child = 2 * node_of + 1 + (xb > nb).long()
        at_level = (node_of >= base) & (node_of < base + L)
        node_of = torch.where(at_level & (nf >= 0), child, node_of)
        alive = alive & (nf >= 0) & at_level if crit == "gini" else (at_level & (nf >= 0))
    return TreeBatch(feature, thr, value, depth)


def _split_search_torch(Xb, stat, feats, local, alive, tot, tt, L, kk, n_bins, crit, lam,
                        min_child):
    """Reference formulation of the split search (CPU path; oracle of tree_hist.hip)."""
    dev = Xb.device
    T, n, _ = stat.shape
    p = Xb.shape[1]
    # histograms: H[t, node, j, bin, 2]
    fsel = torch.gather(feats, 1, local[..., None].expand(T, n, kk))   # [T, n, kk]
    bins = torch.gather(Xb.long()[None].expand(T, n, p), 2, fsel)      # [T, n, kk]
    hidx = ((tt[:, None, None] * L + local[..., None]) * kk +
            torch.arange(kk, device=dev)[None, None]) * n_bins + bins
    H = torch.zeros(T * L * kk * n_bins, 2, device=dev)
    am = alive[..., None].expand(T, n, kk).reshape(-1)
    sv = stat[:, :, None, :].expand(T, n, kk, 2).reshape(-1, 2).float()
    H.index_add_(0, hidx.view(-1)[am], sv[am])
    H = H.view(T, L, kk, n_bins, 2)
    C = torch.cumsum(H, 3)[:, :, :, :-1]                   # left stats for thr = 0..B-2
    Tt = tot[:, :, None, None, :]
    R = Tt - C
    if crit == "gini":
        def gw(s):   # w * gini = w - (wy^2 + (w-wy)^2)/w
            w, wy = s[..., 0], s[..., 1]
            return w - (wy * wy + (w - wy) * (w - wy)) / w.clamp_min(1e-12)
        gain = gw(Tt) - gw(C) - gw(R)
        ok = (C[..., 0] >= 1) & (R[..., 0] >= 1)
    else:
        def sc(s):
            return s[..., 0] * s[..., 0] / (s[..., 1] + lam)
        gain = 0.5 * (sc(C) + sc(R) - sc(Tt))
        ok = (C[..., 1] >= min_child) & (R[..., 1] >= min_child)
    gain = torch.where(ok, gain, torch.full_like(gain, -float("inf")))
    flat = gain.view(T, L, -1)
    best, arg = flat.max(2)
    j = arg // (n_bins - 1)
    b = arg % (n_bins - 1)
    return best, j, b


def grow_sampled(Xb: torch.Tensor, stat: torch.Tensor, depth: int, k: int, n_bins: int,
                 gen: torch.Generator, importance: Optional[torch.Tensor] = None) -> TreeBatch:
    """``grow`` (Gini) with the candidate features drawn inside tree_hist.hip's
    split_search_sampled (k distinct features per node, seeded per level from ``gen``) and up to
    128 bins; stops at the first level where no node splits. Node arrays are stored compact
    (int16 features, uint8 thresholds)."""
    from ..ops.native import lib
    dev = Xb.device
    T, n, _ = stat.shape
    nodes = 2 ** (depth + 1) - 1
    feature = torch.full((T, nodes), -1, dtype=torch.int16, device=dev)
    thr = torch.zeros(T, nodes, dtype=torch.uint8, device=dev)
    value = torch.zeros(T, nodes, device=dev)
    node_of = torch.zeros(T, n, dtype=torch.long, device=dev)
    alive = stat[..., 0] != 0
    tt = torch.arange(T, device=dev)
    stat = stat.float().contiguous()
    used = depth
    for level in range(depth + 1):
        L = 2 ** level
        base = L - 1
        local = (node_of - base).clamp(0, L - 1)
        key = (tt[:, None] * L + local).view(-1)
        tot = torch.zeros(T * L, 2, device=dev)
        m = alive.view(-1)
        tot.index_add_(0, key[m], stat.view(-1, 2)[m])
        tot = tot.view(T, L, 2)
        value[:, base:base + L] = tot[..., 1] / tot[..., 0].clamp_min(1e-12)
        if level == depth:
            break
        nl = torch.where(alive, node_of - base, torch.full_like(node_of, -1)).int().contiguous()
        seed = int(torch.randint(0, 2 ** 62, (1,), generator=gen))
        best, fbest, b = lib().split_search_sampled(Xb, nl, stat, tot.contiguous(), L, k, n_bins,
                                                    0, 1.0, 1.0, seed)
        split = torch.isfinite(best) & (best > 1e-12)
        if not bool(split.any()):
            used = level
            break
        fbest = fbest.long()
        feature[:, base:base + L] = torch.where(split, fbest, torch.full_like(fbest, -1)).to(
            torch.int16)
        thr[:, base:base + L] = b.to(torch.uint8)
        if importance is not None:
            gsum = torch.where(split, best, torch.zeros_like(best))
            importance.index_add_(0, fbest.view(-1), gsum.view(-1).double())
        nf = torch.gather(feature[:, base:base + L], 1, local).long()
        nb = torch.gather(thr[:, base:base + L], 1, local).long()
        xb = Xb[torch.arange(n, device=dev)[None].expand(T, n), nf.clamp_min(0)].long()
        child = 2 * node_of + 1 + (xb > nb).long()
        at_level = (node_of >= base) & (node_of < base + L)
        node_of = torch.where(at_level & (nf >= 0), child, node_of)
        alive = alive & (nf >= 0) & at_level
    return TreeBatch(feature, thr, value, max(used, 1))


class ExactForest:
    """R randomForest on the device: CART with EXACT thresholds (rank bins -- one bin per distinct
    training value, edges at the midpoints; ``exact_bins``), bootstrap counts as sample weights,
    sqrt(p) distinct candidate features per node drawn in the split kernel, grown level by level
    for a chunk of trees at a time until every node is pure or ``max_depth``. MeanDecreaseGini,
    predict and proximity as ``HistForest``. Falls back to 128 quantile bins when a feature has
    more than 128 distinct values (then the thresholds are approximate)."""

    def __init__(self, n_estimators: int = 500, max_depth: int = 13, max_features: str = "sqrt",
                 seed: int = 8, chunk: int = 512):
        self.n, self.depth, self.mf, self.seed, self.chunk = \
            n_estimators, max_depth, max_features, seed, chunk

    def fit(self, X: torch.Tensor, y: torch.Tensor) -> "ExactForest":
        dev = X.device
        n, p = X.shape
        ex = exact_bins(X)
        if ex is None:
            import warnings
            warnings.warn(f"ExactForest: a feature has more than 128 distinct training values "
                          f"(n = {n}); using 128 quantile bins (approximate thresholds)",
                          RuntimeWarning, stacklevel=2)
            Xb, self.edges = quantile_bins(X, 128)
            B = 128
            self.exact = False
        else:
            Xb, self.edges, B = ex
            self.exact = True
        self.n_bins = B
        Xb = Xb.contiguous()
        k = max(1, int(math.sqrt(p))) if self.mf == "sqrt" else (
            max(1, int(math.log2(p))) if self.mf == "log2" else p)
        gen = torch.Generator().manual_seed(self.seed)
        yv = y.float().to(dev)
        self.importance = torch.zeros(p, dtype=torch.float64, device=dev)
        self.batches = []
        self.depth_used = 0
        for s in range(0, self.n, self.chunk):
            T = min(self.chunk, self.n - s)
            draws = torch.randint(0, n, (T, n), generator=gen).to(dev)
            w = torch.zeros(T, n, device=dev)
            w.scatter_add_(1, draws, torch.ones(T, n, device=dev))
            stat = torch.stack([w, w * yv[None]], 2)
            tb = grow_sampled(Xb, stat, self.depth, k, B, gen, importance=self.importance)
            self.depth_used = max(self.depth_used, tb.depth)
            self.batches.append(tb)
        self.mean_decrease_gini = (self.importance / self.n).cpu()
        return self

    def predict_proba(self, X: torch.Tensor) -> torch.Tensor:
        Xb = bin_with(X, self.edges)
        p1 = torch.cat([tb.predict(Xb) for tb in self.batches]).mean(0)
        return torch.stack([1 - p1, p1], 1)

    def predict(self, X: torch.Tensor) -> torch.Tensor:
        return (self.predict_proba(X)[:, 1] > 0.5).long()

    def proximity(self, X: torch.Tensor) -> torch.Tensor:
        """Fraction of trees in which two rows share a leaf ([m, m]), from the leaf ids."""
        Xb = bin_with(X, self.edges)
        m = Xb.shape[0]
        P = torch.zeros(m, m, device=Xb.device)
        for tb in self.batches:
            leaves = tb.apply(Xb)                                      # [T, m]
            P += (leaves[:, :, None] == leaves[:, None, :]).float().sum(0)
        return P / self.n

    @property
    def feature_importances_(self) -> torch.Tensor:
        imp = self.importance.cpu()
        return imp / imp.sum() if imp.sum() > 0 else imp


class HistForest:
    """Random forest: bootstrap counts as sample weights, sqrt(p) features per node, Gini."""

    def __init__(self, n_estimators: int = 500, max_depth: int = 10, max_features: str = "sqrt",
                 n_bins: int = 64, seed: int = 8, chunk: int = 256):
        self.n, self.depth, self.mf, self.bins, self.seed, self.chunk = \
            n_estimators, max_depth, max_features, n_bins, seed, chunk

    def fit(self, X: torch.Tensor, y: torch.Tensor) -> "HistForest":
        dev = X.device
        n, p = X.shape
        self.Xb_edges = None
        Xb, self.edges = quantile_bins(X, self.bins)
        k = max(1, int(math.sqrt(p))) if self.mf == "sqrt" else (
            max(1, int(math.log2(p))) if self.mf == "log2" else p)
        gen = torch.Generator().manual_seed(self.seed)
        yv = y.float().to(dev)
        self.importance = torch.zeros(p, dtype=torch.float64, device=dev)
        self.batches = []
        for s in range(0, self.n, self.chunk):
            T = min(self.chunk, self.n - s)
            draws = torch.randint(0, n, (T, n), generator=gen).to(dev)
            w = torch.zeros(T, n, device=dev)
            w.scatter_add_(1, draws, torch.ones(T, n, device=dev))
            stat = torch.stack([w, w * yv[None]], 2)
            self.batches.append(grow(Xb, stat, self.depth, k, self.bins, "gini", gen=gen,
                                     importance=self.importance))
        self.mean_decrease_gini = (self.importance / self.n).cpu()
        return self

    def predict_proba(self, X: torch.Tensor) -> torch.Tensor:
        Xb = bin_with(X, self.edges)
        p1 = torch.cat([tb.predict(Xb) for tb in self.batches]).mean(0)
        return torch.stack([1 - p1, p1], 1)

    def predict(self, X: torch.Tensor) -> torch.Tensor:
        return (self.predict_proba(X)[:, 1] > 0.5).long()

    def proximity(self, X: torch.Tensor) -> torch.Tensor:
        """randomForest(proximity=TRUE): fraction of trees in which two rows share a leaf
        ([m, m]); accumulated per tree chunk as one-hot(leaf) GEMMs on the device."""
        Xb = bin_with(X, self.edges)
        m = Xb.shape[0]
        P = torch.zeros(m, m, device=Xb.device)
        for tb in self.batches:
            leaves = tb.apply(Xb)                                      # [T, m]
            nodes = tb.feature.shape[1]
            oh = torch.zeros(leaves.shape[0], m, nodes, device=Xb.device)
            oh.scatter_(2, leaves[..., None], 1.0)
            P += torch.einsum("tin,tjn->ij", oh, oh)
        return P / self.n

    @property
    def feature_importances_(self) -> torch.Tensor:
        imp = self.importance.cpu()
        return imp / imp.sum() if imp.sum() > 0 else imp


class HistBoost:
    """Second-order logistic boosting on histogram trees (XGBoost ``tree_method=hist``)."""

    def __init__(self, n_estimators: int = 100, learning_rate: float = 0.3, max_depth: int = 6,
                 reg_lambda: float = 1.0, min_child_weight: float = 1.0, colsample: float = 1.0,
                 n_bins: int = 64, seed: int = 8):
        self.n, self.lr, self.depth, self.lam, self.mcw, self.cs, self.bins, self.seed = \
            n_estimators, learning_rate, max_depth, reg_lambda, min_child_weight, colsample, \
            n_bins, seed

    def fit(self, X: torch.Tensor, y: torch.Tensor) -> "HistBoost":
        dev = X.device
        n, p = X.shape
        Xb, self.edges = quantile_bins(X, self.bins)
        yv = y.float().to(dev)
        margin = torch.zeros(n, device=dev)
        gen = torch.Generator().manual_seed(self.seed)
        self.importance = torch.zeros(p, dtype=torch.float64, device=dev)
        self.trees = []
        for _ in range(self.n):
            pr = torch.sigmoid(margin)
            stat = torch.stack([pr - yv, (pr * (1 - pr)).clamp_min(1e-16)], 1)[None]
            mask = None
            if self.cs < 1:
                kk = max(1, int(round(self.cs * p)))
                mask = torch.zeros(1, p, dtype=torch.bool, device=dev)
                mask[0, torch.randperm(p, generator=gen)[:kk].to(dev)] = True
            tb = grow(Xb, stat, self.depth, p if mask is None else int(mask.sum()), self.bins,
                      "xgb", self.lam, self.mcw, gen, self.importance, mask)
            self.trees.append(tb)
            margin = margin + self.lr * tb.predict(Xb)[0]
        return self

    def predict_proba(self, X: torch.Tensor) -> torch.Tensor:
        Xb = bin_with(X, self.edges)
        m = torch.zeros(X.shape[0], device=X.device)
        for tb in self.trees:
            m = m + self.lr * tb.predict(Xb)[0]
        p1 = torch.sigmoid(m)
        return torch.stack([1 - p1, p1], 1)

    def predict(self, X: torch.Tensor) -> torch.Tensor:
        return (self.predict_proba(X)[:, 1] > 0.5).long()

    @property
    def feature_importances_(self) -> torch.Tensor:
        imp = self.importance.cpu()
        return imp / imp.sum() if imp.sum() > 0 else imp
