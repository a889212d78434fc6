"""Library-size normalisation, TMM and expression filtering (C07), on any torch device.

* ``tmm_factors``  edgeR ``calcNormFactors(method="TMM")`` semantics: reference column by upper
  quartile, per-sample doubly trimmed (30 % log-ratio, 5 % abundance) precision-weighted mean of
  M-values, factors rescaled to geometric mean 1 (`make_seobj_targetaml.R:89-96`).
* ``cpm`` / ``log_cpm``  edgeR ``cpm(..., log=TRUE, prior.count)`` with the library-scaled prior.
* ``filter_by_cpm``  keep genes with CPM >= min_cpm in >= min_samples samples
  (`make_seobj_targetaml.R:90`; the 5 %-of-samples variant of `consensusml_composite.Rmd:510-519`
  via ``min_frac``).
"""
from __future__ import annotations

from typing import Optional

import torch


def lib_sizes(counts: torch.Tensor) -> torch.Tensor:
    return counts.double().sum(0)


def _upper_quartile(x: torch.Tensor) -> torch.Tensor:
    # R quantile type 7 per column
    return torch.quantile(x, 0.75, dim=0)


def _rank_average(v: torch.Tensor) -> torch.Tensor:
    """Ranks 1..n with ties averaged (R's rank default)."""
    s, order = torch.sort(v)
    n = v.numel()
    ranks = torch.empty(n, dtype=torch.float64, device=v.device)
    pos = torch.arange(1, n + 1, dtype=torch.float64, device=v.device)
    uniq, inv, counts = torch.unique_consecutive(s, return_inverse=True, return_counts=True)
    ends = torch.cumsum(counts, 0).double()
    starts = ends - counts.double() + 1
    avg = (starts + ends) / 2
    ranks[order] = avg[inv]
    return ranks


def tmm_factors(counts: torch.Tensor, log_ratio_trim: float = 0.3, sum_trim: float = 0.05,
                weighting: bool = True, a_cutoff: float = -1e10,
                ref_column: Optional[int] = None) -> torch.Tensor:
    """TMM normalisation factors for a genes x samples count matrix (float64 [samples])."""
    x = counts.double()
    lib = x.sum(0)
    if ref_column is None:
        f75 = _upper_quartile(x / lib)
        ref_column = int(torch.argmin((f75 - f75.mean()).abs()))
    ref = x[:, ref_column]
    nR = lib[ref_column]
    facs = torch.empty(x.shape[1], dtype=torch.float64, device=x.device)
    for i in range(x.shape[1]):
        obs = x[:, i]
        nO = lib[i]
        with torch.no_grad():
            logR = torch.log2((obs / nO) / (ref / nR))
            absE = (torch.log2(obs / nO) + torch.log2(ref / nR)) / 2
            v = (nO - obs) / nO / obs + (nR - ref) / nR / ref
        fin = torch.isfinite(logR) & torch.isfinite(absE) & (absE > a_cutoff)
        logR, absE, v = logR[fin], absE[fin], v[fin]
        n = logR.numel()
        if n == 0 or float(logR.abs().max()) < 1e-6:
            facs[i] = 1.0
            continue
        loL = int(n * log_ratio_trim) + 1
        hiL = n + 1 - loL
        loS = int(n * sum_trim) + 1
        hiS = n + 1 - loS
        rL = _rank_average(logR)
        rS = _rank_average(absE)
        keep = (rL >= loL) & (rL <= hiL) & (rS >= loS) & (rS <= hiS)
        if weighting:
            f = (logR[keep] / v[keep]).sum() / (1.0 / v[keep]).sum()
        else:
            f = logR[keep].mean()
        facs[i] = 2.0 ** f if torch.isfinite(f) else 1.0
    return facs / torch.exp(torch.log(facs).mean())


def cpm(counts: torch.Tensor, lib_size: Optional[torch.Tensor] = None) -> torch.Tensor:
    x = counts.double()
    lib = x.sum(0) if lib_size is None else lib_size.double()
    return x / lib * 1e6


def log_cpm(counts: torch.Tensor, lib_size: Optional[torch.Tensor] = None,
            prior_count: float = 1.0) -> torch.Tensor:
    """edgeR log2-CPM: prior scaled by library size, library augmented by 2x the prior."""
    x = counts.double()
    lib = x.sum(0) if lib_size is None else lib_size.double()
    prior = prior_count * lib / lib.mean()
    adj = lib + 2.0 * prior
    return torch.log2((x + prior) / adj * 1e6)


def effective_lib_sizes(counts: torch.Tensor, factors: Optional[torch.Tensor] = None) -> torch.Tensor:
    lib = lib_sizes(counts)
    return lib if factors is None else lib * factors


def filter_by_cpm(counts: torch.Tensor, min_cpm: float = 1.0, min_samples: Optional[int] = 5,
                  min_frac: Optional[float] = None) -> torch.Tensor:
    """Boolean gene mask on the number k of samples with CPM >= min_cpm.

    * ``min_samples`` only: k >= min_samples (make_seobj_targetaml.R:88-91, "in >= 5 samples").
    * ``min_frac`` only: k > min_frac * n, a strict comparison against the non-integer bound,
      exactly ``rowSums(cpm(dge) >= 1) > (0.05*ncol(counts.df))`` of
      JSmith_code/Limma_Voom_DE_Function.R:27 (n = 100 needs 6 samples, not 5).
    * both: both conditions.
    """
    c = cpm(counts)
    n = counts.shape[1]
    k = (c >= min_cpm).sum(1)
    keep = torch.ones_like(k, dtype=torch.bool)
    if min_samples:
        keep &= k >= min_samples
    if min_frac is not None:
        keep &= k.double() > min_frac * n
    return keep


def normalize(es, min_cpm: float = 1.0, min_samples: int = 5, prior_count: float = 1.0):
    """counts -> CPM filter -> TMM -> log-CPM; returns a new ExpressionSet with ``logcpm``
    and the filtered ``counts`` (C07 end to end) plus ``norm_factors`` in col_data."""
    keep = filter_by_cpm(es.assays["counts"], min_cpm, min_samples)
    sub = es.subset(genes=keep.cpu().tolist())
    cnt = sub.assays["counts"]
    f = tmm_factors(cnt)
    lc = log_cpm(cnt, lib_sizes(cnt) * f, prior_count)
    sub.assays["logcpm"] = lc.float()
    cd = sub.col_data.copy()
    if len(cd):
        cd["norm_factors"] = f.cpu().numpy()
        cd["lib_size"] = lib_sizes(cnt).cpu().numpy()
    sub.col_data = cd
    return sub
