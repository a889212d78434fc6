"""Feature-selection consensus (C18, C26) on the same robust-aggregation kernels as the
data-parallel engine.

ConsensusML's "consensus" is agreement of gene sets selected by different models:
pairwise / 3-way set intersections (`scripts/model_walkthrough.ipynb:1846-1939`), a per-gene
membership table, and the **standard output table** — one row per gene (DE statistics first),
one column per model run (`composite_code/rnotebook/cml_targetaml_seanalysis.Rmd:627-633`,
`:679-690`, `:783-799`, `:1075-1091`, `:1246-1263`; artifact `data/standouttable.csv`).

Here each model run contributes an importance vector over the genes; stacking them gives an
[n_models, n_genes] worker matrix, and the robust rules of ``ops.kernels`` give consensus
columns: ``vote`` (how many models selected the gene; vote == n is the n-way intersection),
``median_rank`` / ``trimmed_mean`` of normalised importances, Krum-style outlier-model scores.
When ensemble members run on different ranks, the rows are all-gathered over RCCL first.
"""
from __future__ import annotations

import itertools
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np
import pandas as pd
import torch
import torch.distributed as dist

from ..ops import kernels as K


class StandardTable:
    """Append-only per-gene results table (the reference's ``standtable``)."""

    def __init__(self, genes: Sequence[str], base: Optional[pd.DataFrame] = None):
        self.genes = list(genes)
        self.df = base.copy() if base is not None else pd.DataFrame(index=self.genes)
        if list(self.df.index) != self.genes:
            self.df = self.df.reindex(self.genes)
        self.runs: List[str] = []

    def add(self, name: str, values, genes: Optional[Sequence[str]] = None) -> None:
        """Add one model run's per-gene values; genes not covered get 0 (not NA: the reference
        writes 0 for unselected genes, e.g. lasso coefficients)."""
        if isinstance(values, dict):
            col = pd.Series(0.0, index=self.genes)
            for g, v in values.items():
                if g in col.index:
                    col[g] = float(v)
        else:
            v = values.detach().double().cpu().numpy() if torch.is_tensor(values) else np.asarray(values)
            idx = self.genes if genes is None else list(genes)
            col = pd.Series(0.0, index=self.genes)
            col.loc[idx] = v
        self.df[name] = col.values
        self.runs.append(name)

    def matrix(self, runs: Optional[Sequence[str]] = None) -> torch.Tensor:
        runs = list(runs) if runs is not None else self.runs
        return torch.tensor(self.df[runs].to_numpy(dtype=np.float64).T, dtype=torch.float32)

    def add_consensus(self, runs: Optional[Sequence[str]] = None, thresh: float = 0.0,
                      trim: int = 0, device: Optional[torch.device] = None) -> None:
        """Consensus columns over the model runs: vote count, median |importance| rank score,
        trimmed mean of per-run max-normalised |importance|."""
        runs = list(runs) if runs is not None else list(self.runs)
        X = self.matrix(runs)
        if device is not None:
            X = X.to(device)
        A = X.abs()
        norm = A / A.amax(1, keepdim=True).clamp_min(1e-30)
        # rank score: 1 = most important gene of that run, 0 = unselected
        order = torch.argsort(A, dim=1, descending=True)
        ranks = torch.empty_like(A)
        ar = torch.arange(A.shape[1], device=A.device, dtype=A.dtype)
        ranks.scatter_(1, order, ar.expand_as(A).contiguous())
        score = torch.where(A > thresh, 1.0 - ranks / A.shape[1], torch.zeros_like(A))
        self.df["consensus_votes"] = K.aggregate(torch.ones_like(A) * (A > thresh), "mean")\
            .mul(len(runs)).round().cpu().numpy()
        self.df["consensus_median_rank_score"] = K.aggregate(score, "median").cpu().numpy()
        b = min(trim, (len(runs) - 1) // 2)
        self.df["consensus_trimmed_importance"] = K.aggregate(norm, "trimmed_mean", trim=b)\
            .cpu().numpy()

    def to_csv(self, path: str) -> None:
        """R ``write.csv`` layout (quoted header, row names first, NA for missing) via the
        native runtime's writer when built, pandas otherwise."""
        try:
            from ..runtime import write_csv
            cols = []
            for c in self.df.columns:
                s = self.df[c]
                if s.dtype == object:
                    cols.append((c, [None if pd.isna(v) else str(v) for v in s]))
                else:
                    cols.append((c, [float(v) if pd.notna(v) else float("nan") for v in s]))
            write_csv(path, [str(g) for g in self.genes], cols)
        except ImportError:
            self.df.to_csv(path, na_rep="NA")

    @classmethod
    def read_csv(cls, path: str) -> "StandardTable":
        df = pd.read_csv(path, index_col=0)
        t = cls(list(df.index.astype(str)), df)
        t.runs = [c for c in df.columns if df[c].dtype != object]
        return t


def selected(values, thresh: float = 0.0) -> set:
    """Gene set with |value| > thresh (dict gene -> value, or a pandas Series)."""
    items = values.items() if hasattr(values, "items") else values
    return {g for g, v in items if abs(float(v)) > thresh}


def intersections(sets: Dict[str, set]) -> Dict[str, set]:
    """All pairwise and higher-order intersections, keyed 'a&b', 'a&b&c', ..."""
    out = {}
    names = list(sets)
    for r in range(2, len(names) + 1):
        for combo in itertools.combinations(names, r):
            out["&".join(combo)] = set.intersection(*(sets[c] for c in combo))
    return out


def membership_table(sets: Dict[str, set]) -> pd.DataFrame:
    """Per-gene 0/1 membership in each model's set plus the total count."""
    genes = sorted(set().union(*sets.values())) if sets else []
    df = pd.DataFrame({k: [int(g in s) for g in genes] for k, s in sets.items()}, index=genes)
    df["n_models"] = df.sum(1)
    return df.sort_values("n_models", ascending=False)


def gather_rows(local: torch.Tensor) -> torch.Tensor:
    """All-gather every rank's [k, genes] importance rows (ensemble members as ranks)."""
    if not (dist.is_available() and dist.is_initialized()):
        return local
    out = [torch.empty_like(local) for _ in range(dist.get_world_size())]
    dist.all_gather(out, local.contiguous())
    return torch.cat(out, 0)


def outlier_models(X: torch.Tensor, f: int = 1) -> Dict[str, object]:
    """Krum scores over model importance vectors: models far from the others (a broken run)
    get high scores — the Byzantine view of an ensemble."""
    A = X.float()
    A = A / A.norm(dim=1, keepdim=True).clamp_min(1e-30)
    G = K.gram(A)
    n = A.shape[0]
    sc = torch.zeros(n, dtype=torch.float64, device=A.device)
    w = K.robust_weights(G, "multi_krum", n, f=min(f, max(0, (n - 1) // 2)), m=max(1, n - f),
                         scores=sc)
    return {"scores": sc.cpu(), "kept": (w > 0).cpu()}
