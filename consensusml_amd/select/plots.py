"""Reporting figures (C29, C34): volcano plot, clustered heatmap, importance barplots,
lasso-rep performance curves, correlation-density histograms. matplotlib (Agg) to PNG/JPEG at
the reference's 400 dpi (`composite_code/rnotebook/cml_targetaml_seanalysis.Rmd:578`)."""
from __future__ import annotations

from typing import Dict, Optional, Sequence

import numpy as np
import pandas as pd


def _plt():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt


def volcano(deg: pd.DataFrame, path: str, lfc: float = 1.0, p_cut: float = 0.05,
            label_top: int = 10, dpi: int = 400) -> None:
    """``volcano_plot`` (`...seanalysis.Rmd:317-366`): logFC vs -log10 adj p, labelled top genes."""
    plt = _plt()
    x = deg["logFC"].to_numpy()
    pcol = "p.adj.bh" if "p.adj.bh" in deg else "adj.P.Val"
    y = -np.log10(np.clip(deg[pcol].to_numpy(), 1e-300, 1))
    sig = (np.abs(x) > lfc) & (deg[pcol].to_numpy() < p_cut)
    fig, ax = plt.subplots(figsize=(5, 4))
    ax.scatter(x[~sig], y[~sig], s=4, c="grey")
    ax.scatter(x[sig], y[sig], s=6, c=np.where(x[sig] > 0, "firebrick", "steelblue"))
    for i in np.argsort(-y)[:label_top]:
        ax.annotate(str(deg.index[i])[:15], (x[i], y[i]), fontsize=5)
    ax.axvline(lfc, ls="--", lw=0.5)
    ax.axvline(-lfc, ls="--", lw=0.5)
    ax.axhline(-np.log10(p_cut), ls="--", lw=0.5)
    ax.set_xlabel("log2 fold change")
    ax.set_ylabel("-log10 adjusted p")
    fig.tight_layout()
    fig.savefig(path, dpi=dpi)
    plt.close(fig)


def heatmap(mat: np.ndarray, path: str, row_labels: Optional[Sequence[str]] = None,
            col_groups: Optional[Sequence] = None, dpi: int = 400) -> None:
    """Row-z-scored expression heatmap, columns ordered by group then hierarchical order."""
    from scipy.cluster.hierarchy import leaves_list, linkage
    plt = _plt()
    z = (mat - mat.mean(1, keepdims=True)) / (mat.std(1, keepdims=True) + 1e-12)
    ro = leaves_list(linkage(z, "average")) if z.shape[0] > 2 else np.arange(z.shape[0])
    co = np.arange(z.shape[1])
    if col_groups is not None:
        co = np.argsort(np.asarray(col_groups), kind="stable")
    fig, ax = plt.subplots(figsize=(6, 5))
    ax.imshow(z[ro][:, co], aspect="auto", cmap="RdBu_r", vmin=-3, vmax=3)
    if row_labels is not None and len(row_labels) <= 60:
        ax.set_yticks(range(len(ro)))
        ax.set_yticklabels([row_labels[i] for i in ro], fontsize=4)
    fig.tight_layout()
    fig.savefig(path, dpi=dpi)
    plt.close(fig)


def importance_bars(values: pd.Series, path: str, top: int = 30, dpi: int = 400) -> None:
    plt = _plt()
    v = values.abs().sort_values(ascending=False)[:top]
    fig, ax = plt.subplots(figsize=(5, 4))
    ax.barh(range(len(v))[::-1], v.to_numpy())
    ax.set_yticks(range(len(v))[::-1])
    ax.set_yticklabels([str(i)[:18] for i in v.index], fontsize=5)
    fig.tight_layout()
    fig.savefig(path, dpi=dpi)
    plt.close(fig)


def rep_performance(perf: Dict[str, Sequence[float]], path: str, dpi: int = 400) -> None:
    """TPR / TNR / FDR / FOR across lasso reps (`...seanalysis.Rmd:811-880`)."""
    plt = _plt()
    fig, ax = plt.subplots(figsize=(5, 3.5))
    for k, v in perf.items():
        ax.plot(range(1, len(v) + 1), v, marker="o", label=k)
    ax.set_xlabel("rep")
    ax.legend(fontsize=6)
    fig.tight_layout()
    fig.savefig(path, dpi=dpi)
    plt.close(fig)


def correlation_density(corr: np.ndarray, path: str, dpi: int = 400) -> None:
    plt = _plt()
    iu = np.triu_indices_from(corr, 1)
    fig, ax = plt.subplots(figsize=(4, 3))
    ax.hist(corr[iu], bins=100, density=True)
    ax.set_xlabel("Spearman rho")
    fig.tight_layout()
    fig.savefig(path, dpi=dpi)
    plt.close(fig)
