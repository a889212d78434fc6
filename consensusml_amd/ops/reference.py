"""Pure-PyTorch oracles for every aggregation rule (test oracles + CPU/gloo path).

These are the *definitions* the HIP kernels in ``csrc/kernels`` are checked against
(SURVEY.md §4.4 item 1). Everything here runs on any device in float32/float64 and favours
clarity over speed. There is no reference implementation to mirror: the reference's only
"consensus" is set intersection of per-model feature sets (`scripts/model_walkthrough.ipynb:1939`,
`composite_code/rnotebook/cml_targetaml_seanalysis.Rmd:627-633`), which is the ``vote`` rule below.

Conventions (shared with the kernels):
  * ``X`` is worker-major ``[n, d]``.
  * Non-finite entries sort as +inf in coordinate rules; a worker whose squared norm is
    non-finite gets score +inf / weight 0 in Gram-space rules.
  * Median of an even count is the mean of the two middle values.
  * Gram-space rules return a weight vector ``w`` (sum 1); the aggregate is ``w @ X``.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch

# --------------------------------------------------------------------------- coordinate rules


def _sanitize(X: torch.Tensor) -> torch.Tensor:
    X = X.float()
    return torch.where(torch.isnan(X), torch.full_like(X, float("inf")), X)


def mean(X: torch.Tensor) -> torch.Tensor:
    return X.float().mean(0)


def coord_median(X: torch.Tensor) -> torch.Tensor:
    S, _ = torch.sort(_sanitize(X), dim=0)
    n = S.shape[0]
    if n % 2:
        return S[n // 2]
    return 0.5 * (S[n // 2 - 1] + S[n // 2])


def trimmed_mean(X: torch.Tensor, b: int) -> torch.Tensor:
    n = X.shape[0]
    if 2 * b >= n:
        raise ValueError(f"trimmed_mean needs n > 2b (n={n}, b={b})")
    S, _ = torch.sort(_sanitize(X), dim=0)
    return S[b:n - b].mean(0)


def vote(X: torch.Tensor, thresh: float = 0.0) -> torch.Tensor:
    """Coordinate-wise count of workers with |x| > thresh (ConsensusML's selection consensus:
    count == n is the n-way intersection of `model_walkthrough.ipynb:1939`)."""
    return (X.float().abs() > thresh).sum(0).float()


# --------------------------------------------------------------------------- Gram-space rules


def gram(X: torch.Tensor) -> torch.Tensor:
    Xd = X.double()
    return Xd @ Xd.t()


def sq_dists_from_gram(G: torch.Tensor) -> torch.Tensor:
    d = torch.diagonal(G)
    D = d[:, None] + d[None, :] - 2.0 * G
    return D.clamp_min(0.0)


def _bad_rows(G: torch.Tensor) -> torch.Tensor:
    return ~torch.isfinite(torch.diagonal(G))


def gram_center(G: torch.Tensor) -> int:
    """Medoid of the finite rows (csrc/kernels/gram.hip:gram_center_kernel)."""
    d = torch.diagonal(G)
    ok = torch.isfinite(d)
    D = (d[:, None] + d[None, :] - 2.0 * G).clamp_min(0.0)
    D = torch.where(ok[None, :], D, torch.zeros_like(D))
    s = D.sum(1)
    s = torch.where(ok & torch.isfinite(s), s, torch.full_like(s, float("inf")))
    if not bool(torch.isfinite(s).any()):
        return 0
    best = float(s.min())
    return int(torch.nonzero(s == best)[0, 0])


def krum_scores(G: torch.Tensor, f: int) -> torch.Tensor:
    """score_i = sum of the n-f-2 smallest squared distances from i to the others."""
    n = G.shape[0]
    bad = _bad_rows(G)
    D = sq_dists_from_gram(G)
    D = torch.where(bad[:, None] | bad[None, :], torch.full_like(D, float("inf")), D)
    D = torch.where(torch.isnan(D), torch.full_like(D, float("inf")), D)
    # k = n - f - 2 neighbours, floored at 1 so small pools (Bulyan's last rounds, n = 2f+2)
    # still rank by the nearest neighbour instead of degenerating to index order
    k = min(max(n - f - 2, 1), n - 1)
    scores = torch.zeros(n, dtype=torch.float64, device=G.device)
    for i in range(n):
        others = torch.cat([D[i, :i], D[i, i + 1:]])
        if k > 0:
            scores[i] = torch.sort(others).values[:k].sum()
    scores = torch.where(bad, torch.full_like(scores, float("inf")), scores)
    return scores


def krum_weights(G: torch.Tensor, f: int, m: int = 1) -> torch.Tensor:
    """Krum (m=1) / Multi-Krum (m>1): average of the m lowest-score workers (ties -> lower index)."""
    n = G.shape[0]
    s = krum_scores(G, f)
    idx = sorted(range(n), key=lambda i: (s[i].item(), i))[:m]
    w = torch.zeros(n, dtype=torch.float64, device=G.device)
    w[idx] = 1.0 / m
    return w


def weiszfeld_weights(G: torch.Tensor, iters: int = 8, eps: float = 1e-6,
                      tol: float = 0.0) -> torch.Tensor:
    """Smoothed Weiszfeld entirely in Gram space.

    z_t = sum_j a_j x_j, so ||x_i - z_t||^2 = G_ii - 2 (G a)_i + a^T G a. Each iteration
    sets b_i = 1 / max(||x_i - z_t||, eps), a <- b / sum(b). Starts from the mean.
    """
    n = G.shape[0]
    bad = _bad_rows(G)
    good = (~bad).double()
    Gs = torch.where(bad[:, None] | bad[None, :], torch.zeros_like(G), G)
    a = good / good.sum().clamp_min(1.0)
    for _ in range(iters):
        Ga = Gs @ a
        d2 = (torch.diagonal(Gs) - 2.0 * Ga + a @ Ga).clamp_min(0.0)
        b = good / torch.sqrt(d2).clamp_min(eps)
        a_new = b / b.sum()
        delta = (a_new - a).abs().max().item()
        a = a_new
        if tol > 0 and delta < tol:
            break
    return a


def geomed_direct(X: torch.Tensor, iters: int = 8, eps: float = 1e-6) -> torch.Tensor:
    """Weiszfeld on the raw vectors (independent oracle for the Gram-space version)."""
    Xd = X.double()
    z = Xd.mean(0)
    for _ in range(iters):
        d = torch.sqrt(((Xd - z) ** 2).sum(1)).clamp_min(eps)
        b = 1.0 / d
        z = (b[:, None] * Xd).sum(0) / b.sum()
    return z.float()


def centered_clip_weights(G_aug: torch.Tensor, tau: float, iters: int) -> torch.Tensor:
    """Centered clipping (Karimireddy et al. 2021) in Gram space.

    ``G_aug`` is the (n+1)x(n+1) Gram of [x_1..x_n, v0] where v0 is the previous aggregate.
    v <- v + (1/n) sum_i clip_tau(x_i - v), with v = sum_j c_j y_j over the n+1 rows.
    Workers with a non-finite squared norm are excluded (clip scale 0).
    Returns the n+1 coefficients c (the last multiplies v0).
    """
    n = G_aug.shape[0] - 1
    bad = _bad_rows(G_aug)
    bad[n] = False
    Gs = torch.where(bad[:, None] | bad[None, :], torch.zeros_like(G_aug), G_aug)
    c = torch.zeros(n + 1, dtype=torch.float64, device=G_aug.device)
    c[n] = 1.0
    for _ in range(iters):
        Gc = Gs @ c
        d2 = (torch.diagonal(Gs)[:n] - 2.0 * Gc[:n] + c @ Gc).clamp_min(0.0)
        d = torch.sqrt(d2)
        s = torch.clamp(tau / d.clamp_min(1e-30), max=1.0) / n   # clip scale per worker
        s = torch.where(bad[:n], torch.zeros_like(s), s)
        # v_new = v + sum_i s_i (x_i - v) = (1 - sum s) v + sum s_i x_i
        c_new = c * (1.0 - s.sum())
        c_new[:n] += s
        c = c_new
    return c


def bulyan_select(G: torch.Tensor, f: int) -> torch.Tensor:
    """Bulyan's selection phase: iterated Krum picks theta = n - 2f workers (indices, sorted)."""
    n = G.shape[0]
    theta = n - 2 * f
    remaining = list(range(n))
    chosen = []
    for _ in range(theta):
        sub = G[remaining][:, remaining]
        s = krum_scores(sub, f)
        j = min(range(len(remaining)), key=lambda i: (s[i].item(), i))
        chosen.append(remaining.pop(j))
    return torch.tensor(sorted(chosen), dtype=torch.long)


def bulyan(X: torch.Tensor, f: int) -> torch.Tensor:
    """Bulyan = Krum selection of n-2f workers, then coordinate trimmed mean (trim f)."""
    sel = bulyan_select(gram(X), f)
    return trimmed_mean(X[sel.to(X.device)], f)


# --------------------------------------------------------------------------- full rules


def aggregate(X: torch.Tensor, rule: str, f: int = 0, trim: Optional[int] = None,
              m: Optional[int] = None, iters: int = 8, eps: float = 1e-6,
              tau: float = 10.0, clip_iters: int = 3,
              v0: Optional[torch.Tensor] = None) -> torch.Tensor:
    n = X.shape[0]
    if rule == "mean":
        return mean(X)
    if rule == "median":
        return coord_median(X)
    if rule == "trimmed_mean":
        return trimmed_mean(X, f if trim is None else trim)
    if rule == "krum":
        w = krum_weights(gram(X), f, 1)
        return (w.float() @ _zero_bad(X)).float()
    if rule == "multi_krum":
        w = krum_weights(gram(X), f, m if m is not None else n - f)
        return (w.float() @ _zero_bad(X)).float()
    if rule == "geomed":
        w = weiszfeld_weights(gram(X), iters, eps)
        return (w.float() @ _zero_bad(X)).float()
    if rule == "bulyan":
        return bulyan(X, f)
    if rule == "centered_clip":
        v0 = torch.zeros(X.shape[1], device=X.device) if v0 is None else v0
        Y = torch.cat([X.float(), v0.float()[None]], 0)
        c = centered_clip_weights(gram(Y), tau, clip_iters)
        return (c.float() @ _zero_bad(Y)).float()
    raise ValueError(f"unknown rule {rule!r}")


def _zero_bad(X: torch.Tensor) -> torch.Tensor:
    X = X.float()
    ok = torch.isfinite(X).all(1, keepdim=True)
    return torch.where(ok, X, torch.zeros_like(X))


# --------------------------------------------------------------------------- optimizers


def sgd_update(p: torch.Tensor, g: torch.Tensor, buf: torch.Tensor, lr: float, momentum: float,
               weight_decay: float = 0.0, nesterov: bool = False, first: bool = False
               ) -> Tuple[torch.Tensor, torch.Tensor]:
    """torch.optim.SGD semantics on fp32 master ``p`` and momentum ``buf`` (returns new copies)."""
    g = g.float()
    if weight_decay:
        g = g + weight_decay * p
    if momentum:
        buf = g.clone() if first else momentum * buf + g
        g = g + momentum * buf if nesterov else buf
    return p - lr * g, buf


def adam_update(p, g, m, v, step: int, lr: float, beta1: float, beta2: float, eps: float,
                weight_decay: float = 0.0, decoupled: bool = True):
    g = g.float()
    if weight_decay and not decoupled:
        g = g + weight_decay * p
    if weight_decay and decoupled:
        p = p * (1.0 - lr * weight_decay)
    m = beta1 * m + (1 - beta1) * g
    v = beta2 * v + (1 - beta2) * g * g
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = (v / bc2).sqrt() + eps
    p = p - (lr / bc1) * m / denom
    return p, m, v


def gossip_mix(x: torch.Tensor, left: torch.Tensor, right: torch.Tensor, w0: float, w1: float,
               w2: float, clip: float = 0.0) -> torch.Tensor:
    x = x.float()
    dl = left.float() - x
    dr = right.float() - x
    if clip > 0:
        nl = dl.norm().item()
        nr = dr.norm().item()
        dl = dl * min(1.0, clip / max(nl, 1e-30))
        dr = dr * min(1.0, clip / max(nr, 1e-30))
    # w0 x + w1 (x + dl) + w2 (x + dr)
    return (w0 + w1 + w2) * x + w1 * dl + w2 * dr


def gossip_mix_k(x: torch.Tensor, nbrs, w, w0: float, clip: float = 0.0) -> torch.Tensor:
    """x <- (w0 + sum w_k) x + sum_k w_k c_k (nb_k - x), c_k = min(1, clip / ||nb_k - x||)."""
    x = x.float()
    out = (w0 + sum(w)) * x
    for nb, wk in zip(nbrs, w):
        d = nb.float() - x
        if clip > 0:
            d = d * min(1.0, clip / max(d.norm().item(), 1e-30))
        out = out + wk * d
    return out


def ceil_div(a: int, b: int) -> int:
    return -(-a // b)


def is_pow2(n: int) -> bool:
    return n > 0 and (n & (n - 1)) == 0


__all__ = [n for n in dir() if not n.startswith("_") and n not in ("math", "torch", "Optional",
                                                                     "Tuple", "annotations")]
