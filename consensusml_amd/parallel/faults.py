"""Byzantine fault injection (N10): corrupt selected workers' local gradients before exchange.

Elementwise attacks (sign flip, Gaussian, scaling, zero, NaN) run as one HIP kernel on GPU
(``ops.inject_fault``). Collusion attacks need honest statistics:
  * ALIE ("A Little Is Enough", Baruch et al. 2019): x = mu - z * sigma (coordinate-wise)
  * IPM  (inner-product manipulation, Xie et al. 2020): x = -scale * mu
where mu / sigma are over the honest workers. In the distributed engine the colluders obtain them
with one extra all-reduce of (sum, sum of squares, count) — simulation cost only, paid only when
such an attack is configured.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from ..config import FaultConfig
from ..ops.kernels import inject_fault

ELEMENTWISE = ("sign_flip", "gaussian", "scaled", "zero", "nan")
COLLUSION = ("alie", "ipm")


def byzantine_rows(cfg: FaultConfig, rank: int, rows_per_rank: int, step: int) -> List[int]:
    """Local gradient rows (virtual workers of this rank) that are Byzantine at ``step``."""
    if cfg.kind == "none" or step < cfg.start_step:
        return []
    base = rank * rows_per_rank
    return [w - base for w in cfg.ranks if base <= w < base + rows_per_rank]


def apply_faults(G: torch.Tensor, cfg: FaultConfig, rank: int, step: int,
                 group_active: bool, seed: int = 0, cols: Optional[slice] = None) -> None:
    """Corrupt rows of the local gradient matrix ``G`` ([rows, D]) in place.

    ``cols`` restricts the attack to a column range (bucket-wise injection during backward).
    ``group_active``: a process group exists (collusion statistics are all-reduced).
    """
    rows = G.shape[0]
    bad = byzantine_rows(cfg, rank, rows, step)
    if cfg.kind == "none" or step < cfg.start_step:
        return
    sl = cols if cols is not None else slice(None)
    if cfg.kind in ELEMENTWISE:
        # bucket-wise injection (overlap / early update): the column offset enters the seed so
        # every bucket gets its own noise stream instead of a repeat of the first one
        col0 = (cols.start or 0) if cols is not None else 0
        for r in bad:
            g = G[r, sl]
            sd = seed * 1000003 + rank * 131 + r + col0 * 7919
            if not g.is_contiguous():
                tmp = g.contiguous()
                inject_fault(tmp, cfg.kind, cfg.scale, cfg.sigma, sd)
                g.copy_(tmp)
            else:
                inject_fault(g, cfg.kind, cfg.scale, cfg.sigma, sd)
        return
    if cfg.kind in COLLUSION:
        honest = [r for r in range(rows) if r not in bad]
        X = G[:, sl].float()
        if honest:
            H = X[honest]
            s1 = H.sum(0)
            s2 = (H * H).sum(0)
            cnt = torch.tensor([float(len(honest))], device=G.device)
        else:
            s1 = torch.zeros(X.shape[1], device=G.device)
            s2 = torch.zeros_like(s1)
            cnt = torch.zeros(1, device=G.device)
        if group_active:
            dist.all_reduce(s1)
            dist.all_reduce(s2)
            dist.all_reduce(cnt)
        mu = s1 / cnt.clamp_min(1)
        var = (s2 / cnt.clamp_min(1) - mu * mu).clamp_min(0)
        if cfg.kind == "alie":
            evil = mu - cfg.z * var.sqrt()
        else:
            evil = -cfg.scale * mu
        for r in bad:
            G[r, sl] = evil.to(G.dtype)
        return
    raise ValueError(f"unknown fault kind {cfg.kind!r}")
