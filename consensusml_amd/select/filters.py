"""Feature pre-filters and data splits (C12, C13, C14, C19, RYAN's mean-difference filter).

* ``seeded_split``        2/3 train split of patients with a seed (`JSmith_code/Differential_
                          Expression_and_Lasso.Rmd:158-187`), persisted as CSV id lists.
* ``variance_filter``     top (or bottom) k most variable genes within each class, unioned
                          (``data_prep_columns``, `scripts/model_comp.py:37-80`).
* ``holdout_split``       20 % holdout then a 67/33 train/test split (``model_prep``,
                          `scripts/model_comp.py:82-121`).
* ``random_genes``        random-gene negative control (`model_walkthrough.ipynb:1245`).
* ``mean_difference_filter``  |mean(class1) - mean(class0)| > delta (`Ryan/Feature_selection_
                          GLMTrain_WT_TARGET.R:44-52`).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch


def seeded_split(ids: Sequence[str], frac: float = 2 / 3, seed: int = 2019) -> Tuple[List[str], List[str]]:
    g = np.random.default_rng(seed)
    ids = list(ids)
    k = int(round(frac * len(ids)))
    pick = set(g.choice(len(ids), k, replace=False).tolist())
    train = [s for i, s in enumerate(ids) if i in pick]
    test = [s for i, s in enumerate(ids) if i not in pick]
    return train, test


def write_split(train: Sequence[str], test: Sequence[str], prefix: str) -> None:
    import pandas as pd
    pd.DataFrame({"x": list(train)}).to_csv(prefix + "_Training_Samples.csv")
    pd.DataFrame({"x": list(test)}).to_csv(prefix + "_Testing_Samples.csv")


def variance_filter(X: torch.Tensor, y: torch.Tensor, k: int = 1000, largest: bool = True) -> torch.Tensor:
    """Union over classes of each class's k highest- (or lowest-) variance feature columns.
    X [samples, genes]; returns sorted column indices."""
    cols = []
    for c in torch.unique(y):
        Xc = X[y == c].double()
        v = Xc.var(0) if Xc.shape[0] > 1 else torch.zeros(X.shape[1], dtype=torch.float64)
        kk = min(k, X.shape[1])
        cols.append(torch.topk(v, kk, largest=largest).indices)
    return torch.unique(torch.cat(cols)).sort().values


def holdout_split(n: int, holdout_frac: float = 0.2, test_frac: float = 0.33, seed: int = 8):
    """(train_idx, test_idx, holdout_idx) — holdout first, then train/test on the rest."""
    g = np.random.default_rng(seed)
    perm = g.permutation(n)
    h = int(round(holdout_frac * n))
    hold, rest = perm[:h], perm[h:]
    t = int(np.ceil(test_frac * rest.size))
    rest = g.permutation(rest)
    return np.sort(rest[t:]), np.sort(rest[:t]), np.sort(hold)


def random_genes(n_genes: int, k: int = 2000, seed: int = 0) -> np.ndarray:
    return np.sort(np.random.default_rng(seed).choice(n_genes, min(k, n_genes), replace=False))


def mean_difference_filter(X: torch.Tensor, y: torch.Tensor, delta: float = 0.05) -> torch.Tensor:
    d = (X[y == 1].double().mean(0) - X[y == 0].double().mean(0)).abs()
    return torch.nonzero(d > delta).flatten()
