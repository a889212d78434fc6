"""Device-dispatching wrappers of the aggregation / optimizer / gossip kernels.

GPU tensors -> HIP kernels of ``csrc/kernels`` (via ``_C``); CPU tensors -> the oracles of
``ops.reference`` (used by the gloo plumbing config and the CPU tests). Worker matrices are
``[n, D]`` worker-major with unit column stride (row stride free, so views into all-gather /
all-to-all receive buffers need no copy).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch

from . import reference as ref
from .native import lib

RULE_IDS = {"mean": 0, "krum": 1, "multi_krum": 2, "geomed": 3, "centered_clip": 4,
            "bulyan_select": 5}
COORD_RULES = ("median", "trimmed_mean")
GRAM_RULES = ("krum", "multi_krum", "geomed", "centered_clip")
GOSSIP_MAX_NBRS = 8   # neighbour buffers one gossip_mix_k launch reads (kMaxNbrs, gossip_fault.hip)


def sorted_range(rule: str, n: int, trim: int = 0) -> Tuple[int, int]:
    """Sorted-rank window [lo, lo+cnt) averaged by a coordinate rule over n values."""
    if rule == "median":
        return ((n - 1) // 2, 1) if n % 2 else (n // 2 - 1, 2)
    if rule == "trimmed_mean":
        if 2 * trim >= n:
            raise ValueError(f"trimmed_mean needs n > 2*trim (n={n}, trim={trim})")
        return trim, n - 2 * trim
    if rule == "mean":
        return 0, n
    raise ValueError(rule)


@dataclass
class OptArgs:
    """Hyper-parameters of one fused optimizer step (SGD or Adam/AdamW)."""
    kind: str = "sgd"            # none | sgd | adam (L2 weight decay) | adamw (decoupled)
    lr: float = 0.1
    momentum: float = 0.0
    weight_decay: float = 0.0
    nesterov: bool = False
    first: bool = False          # first SGD step: momentum buffer <- g
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = 1e-8
    step: int = 1                # Adam step (1-based) for bias correction
    gscale: float = 1.0

    def opt_id(self) -> int:
        return {"none": 0, "sgd": 1, "adamw": 2, "adam": 3 if self.weight_decay else 2}[self.kind]


def _as2d(X: torch.Tensor) -> torch.Tensor:
    if X.dim() == 1:
        X = X[None]
    assert X.dim() == 2 and X.stride(1) == 1, "worker matrix must be [n, D] with unit column stride"
    return X


# --------------------------------------------------------------------------- fused update
def agg_update(X: torch.Tensor, *, combine: str, lo: int = 0, cnt: int = 1,
               w: Optional[torch.Tensor] = None, rows: Optional[torch.Tensor] = None,
               n: Optional[int] = None, D: Optional[int] = None, opt: Optional[OptArgs] = None,
               master: Optional[torch.Tensor] = None, s1: Optional[torch.Tensor] = None,
               s2: Optional[torch.Tensor] = None, param_out: Optional[torch.Tensor] = None,
               gout: Optional[torch.Tensor] = None) -> None:
    """Aggregate worker rows and apply the optimizer in one pass (in place on the state).

    combine='sorted'   mean of sorted ranks [lo, lo+cnt) per coordinate
    combine='weighted' sum_i w_i x_i (w None -> all ones)
    """
    X = _as2d(X)
    n = n if n is not None else (rows.numel() if rows is not None else X.shape[0])
    D = D if D is not None else X.shape[1]
    opt = opt or OptArgs(kind="none")
    if X.is_cuda:
        bc1 = 1.0 - opt.beta1 ** opt.step
        bc2 = 1.0 - opt.beta2 ** opt.step
        lib().agg_update(X, n, D, rows, 0 if combine == "sorted" else 1, lo, cnt, w, opt.opt_id(),
                         master, s1, s2, param_out, gout, opt.lr, opt.momentum, opt.weight_decay,
                         opt.beta1, opt.beta2, opt.eps, opt.lr / bc1, 1.0 / math.sqrt(bc2),
                         opt.gscale, opt.nesterov, opt.first)
        return
    # ---- CPU reference path
    Xr = X[rows.long()] if rows is not None else X[:n]
    Xr = Xr[:, :D].float()
    if combine == "sorted":
        S, _ = torch.sort(ref._sanitize(Xr), dim=0)
        g = S[lo:lo + cnt].mean(0)
    else:
        ww = torch.ones(n) if w is None else w[:n].float().cpu()
        nz = (ww != 0).nonzero().flatten()
        g = (ww[nz, None] * Xr[nz]).sum(0) if nz.numel() else torch.zeros(D)
    g = g * opt.gscale
    if gout is not None:
        gout[:D].copy_(g)
    k = opt.opt_id()
    if k == 0:
        return
    if k == 1:
        p, b = ref.sgd_update(master[:D], g, s1[:D] if s1 is not None else None, opt.lr,
                              opt.momentum, opt.weight_decay, opt.nesterov, opt.first)
        master[:D].copy_(p)
        if opt.momentum:
            s1[:D].copy_(b)
    else:
        p, m, v = ref.adam_update(master[:D], g, s1[:D], s2[:D], opt.step, opt.lr, opt.beta1,
                                  opt.beta2, opt.eps, opt.weight_decay, decoupled=(k == 2))
        master[:D].copy_(p)
        s1[:D].copy_(m)
        s2[:D].copy_(v)
    if param_out is not None:
        param_out[:D].copy_(master[:D].to(param_out.dtype))


# --------------------------------------------------------------------------- Gram + weights
class GramWorkspace:
    """Per-device cache of the split-K partial buffer of the Gram kernel."""
    _cache = {}

    @classmethod
    def get(cls, device: torch.device, n: int, D: int) -> torch.Tensor:
        nbytes = lib().gram_workspace_bytes(n, D)
        key = (device, nbytes)
        buf = cls._cache.get(key)
        if buf is None:
            buf = torch.empty(nbytes // 4, dtype=torch.float32, device=device)
            cls._cache[key] = buf
        return buf


def agg_update_multi(segs, *, combine: str, lo: int = 0, cnt: int = 1,
                     w: Optional[torch.Tensor] = None, rows: Optional[torch.Tensor] = None,
                     n: int, opt: Optional[OptArgs] = None, master: Optional[torch.Tensor] = None,
                     s1: Optional[torch.Tensor] = None, s2: Optional[torch.Tensor] = None,
                     gout: Optional[torch.Tensor] = None) -> None:
    """``agg_update`` over several segments in ONE launch on GPU (the sharded engine's buckets).
    ``segs``: (X [rows, >= D], D, off, param_out) -- worker rows, element count, offset into the
    shared master / s1 / s2 / gout vectors, and the segment's parameters."""
    opt = opt or OptArgs(kind="none")
    if segs and segs[0][0].is_cuda and len(segs) <= 16:
        bc1 = 1.0 - opt.beta1 ** opt.step
        bc2 = 1.0 - opt.beta2 ** opt.step
        lib().agg_update_multi([_as2d(x) for x, _, _, _ in segs], [int(d) for _, d, _, _ in segs],
                               [int(o) for _, _, o, _ in segs], [p for _, _, _, p in segs], n,
                               rows, 0 if combine == "sorted" else 1, lo, cnt, w, opt.opt_id(),
                               master, s1, s2, gout, opt.lr, opt.momentum, opt.weight_decay,
                               opt.beta1, opt.beta2, opt.eps, opt.lr / bc1, 1.0 / math.sqrt(bc2),
                               opt.gscale, opt.nesterov, opt.first)
        return
    sl = lambda t, o, d: None if t is None else t[o:o + d]   # noqa: E731
    for X, D, off, pout in segs:
        agg_update(X, combine=combine, lo=lo, cnt=cnt, w=w, rows=rows, n=n, D=D, opt=opt,
                   master=sl(master, off, D), s1=sl(s1, off, D), s2=sl(s2, off, D),
                   param_out=pout, gout=sl(gout, off, D))


def gram(X: torch.Tensor, rows: Optional[torch.Tensor] = None, n: Optional[int] = None,
         D: Optional[int] = None, out: Optional[torch.Tensor] = None,
         accumulate: bool = False, center: Optional[torch.Tensor] = None) -> torch.Tensor:
    """G = X X^T in fp64 ([n, n]); MFMA kernel on GPU. ``accumulate``: out += X X^T.
    ``center`` (int32 [1] on X's device): the Gram of the rows relative to row ``center[0]``
    (same distances, no cancellation for near-duplicate rows; see ``gram_center``)."""
    X = _as2d(X)
    n = n if n is not None else (rows.numel() if rows is not None else X.shape[0])
    D = D if D is not None else X.shape[1]
    if X.is_cuda:
        if out is None:
            out = torch.empty(n, n, dtype=torch.float64, device=X.device)
        if X.data_ptr() % 16 or (X.stride(0) * X.element_size()) % 16:
            X = X[:n if rows is None else X.shape[0], :D].contiguous()
            X = torch.nn.functional.pad(X, (0, (-D) % 8))
        if accumulate and out is None:
            raise ValueError("accumulate needs out")
        ws = GramWorkspace.get(X.device, n, D)
        lib().gram(X, n, D, rows, ws, out, accumulate, center)
        return out
    Xr = X[rows.long()] if rows is not None else X[:n]
    Xr = Xr[:, :D]
    if center is not None and int(center[0]) >= 0:   # a negative center: uncentered pass
        c = min(int(center[0]), n - 1)
        xc = Xr[c].double()
        Xr = Xr.double() - torch.where(torch.isfinite(xc), xc, torch.zeros_like(xc))
    G = ref.gram(Xr)
    if out is not None:
        if accumulate:
            out.add_(G)
        else:
            out.copy_(G)
        return out
    return G


def gram_center(G: torch.Tensor, n: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """int32 [1]: the medoid of the finite rows of G (least summed squared distance to the
    other finite rows; ties -> lower index), the center of a second, centered Gram pass."""
    if out is None:
        out = torch.zeros(1, dtype=torch.int32, device=G.device)
    if G.is_cuda:
        lib().gram_center(G.contiguous(), n, out)
        return out
    out.reshape(-1)[0] = ref.gram_center(G[:n, :n])   # (element 1 of an engine center: guard state)
    return out


def gram_sum(Gb: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out = Gb[0] + Gb[1] + ... in bucket order (one launch on GPU; the same fp64 adds as
    accumulating the buckets' Grams one after another)."""
    if Gb.is_cuda:
        lib().gram_sum(Gb, out)
        return out
    out.copy_(Gb[0])
    for k in range(1, Gb.shape[0]):
        out.add_(Gb[k])
    return out


def robust_weights(G: torch.Tensor, rule: str, n: int, f: int = 0, m: Optional[int] = None,
                   iters: int = 8, eps: float = 1e-6, tol: float = 0.0, tau: float = 10.0,
                   w_out: Optional[torch.Tensor] = None, scores: Optional[torch.Tensor] = None,
                   sel: Optional[torch.Tensor] = None, guard: bool = False,
                   center_out: Optional[torch.Tensor] = None,
                   sel_counts: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Weights over worker rows (fp32 [n] or [n+1] for centered clipping) from the Gram matrix.

    In the same launch (weights.hip): ``sel_counts`` += (w > 0); ``center_out`` = the medoid of
    G (the next step's Gram center); ``guard`` (G from a pass centered on the previous step's
    medoid): at least half the worker rows non-finite = a captured center -> weights zeroed
    (centered clipping keeps its previous aggregate) and ``center_out`` = -1. ``center_out``
    holds, on entry, the center this pass used: a negative one (an uncentered pass, e.g. the step
    after a trip) disarms the guard; a 2-element ``center_out`` also carries the previous pass's
    count of non-finite rows, and only an increase trips -- so workers that are genuinely
    non-finite (even half of them) are aggregated around instead of freezing the weights."""
    dim = n + 1 if rule == "centered_clip" else n
    if G.is_cuda:
        if w_out is None:
            w_out = torch.empty(dim, dtype=torch.float32, device=G.device)
        lib().robust_weights(G.contiguous(), RULE_IDS[rule], n, f, m or 0, iters, eps, tol, tau,
                             w_out, scores, sel, guard, center_out, sel_counts)
        return w_out
    if guard and center_out is not None and int(center_out.reshape(-1)[0]) < 0:
        guard = False
    w = _robust_weights_ref(G, rule, n, f, m, iters, eps, tol, tau, scores, sel)
    nbad = int((~torch.isfinite(torch.diagonal(G)[:n])).sum())
    trip = guard and nbad > 0 and 2 * nbad >= n
    if center_out is not None and center_out.numel() >= 2:
        # element 1: the previous pass's non-finite row count (only an INCREASE trips)
        trip = trip and nbad > int(center_out.reshape(-1)[1])
        center_out.reshape(-1)[1] = nbad
    if trip:
        w = torch.zeros_like(w)
        if rule == "centered_clip":
            w[n] = 1.0
        if sel is not None and rule != "bulyan_select":
            sel[:n].zero_()
    if sel_counts is not None:
        sel_counts += (w[:n] > 0).double()
    if center_out is not None:
        center_out.reshape(-1)[0] = -1 if trip else ref.gram_center(G[:n, :n])
    if w_out is not None:
        w_out.copy_(w)
        return w_out
    return w


def _robust_weights_ref(G, rule, n, f, m, iters, eps, tol, tau, scores, sel) -> torch.Tensor:
    if rule == "mean":
        bad = ~torch.isfinite(torch.diagonal(G))
        good = (~bad).double()
        w = good / good.sum().clamp_min(1)
    elif rule == "krum":
        w = ref.krum_weights(G, f, 1)
        if scores is not None:
            scores.copy_(ref.krum_scores(G, f))
    elif rule == "multi_krum":
        w = ref.krum_weights(G, f, m if m else n - f)
        if scores is not None:
            scores.copy_(ref.krum_scores(G, f))
    elif rule == "geomed":
        w = ref.weiszfeld_weights(G, iters, eps, tol)
    elif rule == "centered_clip":
        w = ref.centered_clip_weights(G, tau, iters)
    elif rule == "bulyan_select":
        idx = ref.bulyan_select(G, f)
        w = torch.zeros(n, dtype=torch.float64)
        w[idx] = 1.0 / idx.numel()
        if sel is not None:
            sel[: idx.numel()] = idx.to(sel.dtype)
            sel[n] = idx.numel()
    else:
        raise ValueError(rule)
    if sel is not None and rule != "bulyan_select":
        sel[:n].copy_((w[:n] > 0).to(sel.dtype))
    return w.float()


# --------------------------------------------------------------------------- high level
def aggregate(X: torch.Tensor, rule: str, f: int = 0, trim: Optional[int] = None,
              m: Optional[int] = None, iters: int = 8, eps: float = 1e-6, tau: float = 10.0,
              clip_iters: int = 3, v0: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Full robust aggregate of a local [n, D] worker matrix -> fp32 [D] (native on GPU)."""
    X = _as2d(X)
    n, D = X.shape
    out = torch.empty(D, dtype=torch.float32, device=X.device)
    if rule in ("mean",):
        agg_update(X, combine="weighted", w=torch.full((n,), 1.0 / n, device=X.device), gout=out)
    elif rule in COORD_RULES:
        lo, cnt = sorted_range(rule, n, f if trim is None else trim)
        agg_update(X, combine="sorted", lo=lo, cnt=cnt, gout=out)
    elif rule in ("krum", "multi_krum", "geomed"):
        G = gram(X)
        w = robust_weights(G, rule, n, f, m, iters, eps)
        agg_update(X, combine="weighted", w=w, gout=out)
    elif rule == "centered_clip":
        v0 = torch.zeros(D, dtype=X.dtype, device=X.device) if v0 is None else v0.to(X.dtype)
        Y = torch.cat([X, v0[None]], 0)
        G = gram(Y)
        c = robust_weights(G, "centered_clip", n, tau=tau, iters=clip_iters)
        # non-finite workers carry weight 0 and are skipped by the weighted kernel
        agg_update(Y, combine="weighted", w=c, n=n + 1, gout=out)
    elif rule == "bulyan":
        G = gram(X)
        sel = torch.zeros(n + 1, dtype=torch.int32, device=X.device)
        robust_weights(G, "bulyan_select", n, f, sel=sel)
        theta = n - 2 * f
        lo, cnt = sorted_range("trimmed_mean", theta, f)
        agg_update(X, combine="sorted", lo=lo, cnt=cnt, rows=sel[:theta], n=theta, gout=out)
    else:
        raise ValueError(f"unknown rule {rule!r}")
    return out


def gossip_mix(master: torch.Tensor, left: torch.Tensor, right: torch.Tensor, w0: float,
               w1: float, w2: float, clip: float = 0.0,
               param_out: Optional[torch.Tensor] = None,
               work: Optional[torch.Tensor] = None) -> None:
    """In-place ring mixing of the fp32 master with the neighbours' bf16 parameters."""
    if master.is_cuda:
        if work is None:
            work = torch.empty(lib().gossip_workspace_bytes(master.numel()) // 4,
                               dtype=torch.float32, device=master.device)
        lib().gossip_mix(master, param_out, left, right, w0, w1, w2, clip, work)
        return
    x = ref.gossip_mix(master, left, right, w0, w1, w2, clip)
    master.copy_(x)
    if param_out is not None:
        param_out.copy_(x.to(param_out.dtype))


def gossip_mix_k(master: torch.Tensor, nbrs: List[torch.Tensor], w: List[float], w0: float,
                 clip: float = 0.0, param_out: Optional[torch.Tensor] = None,
                 work: Optional[torch.Tensor] = None,
                 param_out2: Optional[torch.Tensor] = None) -> None:
    """In-place k-neighbour mixing (1 <= k <= 8) of the fp32 master with the neighbours' bf16
    parameters: x <- (w0 + sum w_k) x + sum_k w_k clip_k(nb_k - x). ``param_out2``: a second
    copy of the rounded parameters (the delayed-gossip send buffer) written in the same pass."""
    if master.is_cuda:
        if work is None:
            work = torch.empty(lib().gossip_workspace_bytes(master.numel()) // 4,
                               dtype=torch.float32, device=master.device)
        lib().gossip_mix_k(master, param_out, list(nbrs), [float(v) for v in w], w0, clip, work,
                           param_out2)
        return
    x = ref.gossip_mix_k(master, nbrs, w, w0, clip)
    master.copy_(x)
    if param_out is not None:
        param_out.copy_(x.to(param_out.dtype))
    if param_out2 is not None:
        param_out2.copy_(x.to(param_out2.dtype))


FAULT_IDS = {"none": 0, "sign_flip": 1, "gaussian": 2, "scaled": 3, "zero": 4, "nan": 5}


def inject_fault(g: torch.Tensor, kind: str, scale: float = 10.0, sigma: float = 1.0,
                 seed: int = 0) -> None:
    """Corrupt a local flat gradient in place (Byzantine simulation)."""
    if kind == "none":
        return
    if g.is_cuda and kind in FAULT_IDS:
        lib().fault(g, FAULT_IDS[kind], scale, sigma, seed)
        return
    if kind == "sign_flip":
        g.mul_(-scale)
    elif kind == "gaussian":
        gen = torch.Generator(device=g.device).manual_seed(seed)
        g.copy_(torch.randn(g.shape, generator=gen, device=g.device) * sigma)
    elif kind == "scaled":
        g.mul_(scale)
    elif kind == "zero":
        g.zero_()
    elif kind == "nan":
        g.fill_(float("nan"))
    else:
        raise ValueError(f"fault {kind!r} needs cross-worker statistics (see parallel.faults)")
