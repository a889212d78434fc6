"""End-to-end feature-selection consensus pipeline (reference call stack SURVEY.md §3.2 / §3.3).

``consensus_pipeline`` mirrors `composite_code/rnotebook/cml_targetaml_seanalysis.Rmd` end to end:
normalise -> DE genes on the training split -> standard table seeded with DE statistics ->
4 SVM runs (linear / radial x weight filter) -> iterative-exclusion lasso reps -> random forests
-> boosted trees -> consensus columns -> CSV + JSON summary. Defects of the reference are not
reproduced (§4.3): every rep's coefficients are kept, SVM weights come from the refit model, tree
metrics use the current model's predictions.

Ensemble parallelism: the model runs ("members") are independent, so with a process group each
rank runs members[rank::world] and the per-gene importance vectors are all-gathered — the same
"workers as ranks" structure as the data-parallel engine.
"""
from __future__ import annotations

import json
import os
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import pandas as pd
import torch
import torch.distributed as dist

from .consensus import StandardTable, intersections, membership_table, selected
from .data import ExpressionSet
from .de import voom_de
from .lasso import iterative_exclusion
from .metrics import binary_metrics
from .normalize import normalize
from .svm import run_svm
from .hist_trees import HistBoost, HistForest

Member = Tuple[str, Callable[[], Dict[str, object]]]


def _run_members(members: List[Member]) -> Dict[str, Dict[str, object]]:
    """Run members (sharded over ranks when a process group exists) and gather their
    {'values': {gene: v} or array, 'metrics': {...}} results on every rank."""
    rank, world = 0, 1
    if dist.is_available() and dist.is_initialized():
        rank, world = dist.get_rank(), dist.get_world_size()
    mine = {}
    for i, (name, fn) in enumerate(members):
        if i % world == rank:
            mine[name] = fn()
    if world == 1:
        return mine
    gathered: List[Optional[dict]] = [None] * world
    dist.all_gather_object(gathered, mine)
    out = {}
    for d in gathered:
        out.update(d)
    return {name: out[name] for name, _ in members}


def consensus_pipeline(es: ExpressionSet, label_col: str = "low_risk",
                       split_col: str = "exptset", out_dir: Optional[str] = None,
                       seed: int = 2019, lasso_reps: int = 3, rf_trees: Sequence[int] = (200, 500),
                       xgb_configs: Sequence[dict] = ({"max_depth": 2, "n_estimators": 2},
                                                      {"max_depth": 6, "n_estimators": 50}),
                       de_lfc: float = 1.0, device: Optional[torch.device] = None,
                       max_genes: Optional[int] = None) -> Dict[str, object]:
    dev = device or torch.device("cpu")
    if "logcpm" not in es.assays:
        es = normalize(es)
    y_all = torch.as_tensor(es.col_data[label_col].to_numpy(), dtype=torch.long)
    train = np.where(es.col_data[split_col].to_numpy() == "train")[0]
    test = np.where(es.col_data[split_col].to_numpy() == "test")[0]

    # ---------------------------------------------------------------- DE genes on training split
    cnt = es.assays["counts"]
    deg = voom_de(cnt[:, train], y_all[train].tolist(), es.genes, lfc=de_lfc)
    genes = list(deg.index)
    if max_genes is not None:
        genes = genes[:max_genes]
    if len(genes) < 2:
        raise RuntimeError("fewer than 2 differentially expressed genes")
    sub = es.subset(genes=genes)
    X = sub.assays["logcpm"].t().contiguous().float().to(dev)          # samples x genes
    y = y_all.to(dev)
    table = StandardTable(genes, deg.loc[genes].rename(columns={"P.Value": "p.unadj",
                                                               "adj.P.Val": "p.adj.bh"}))
    Xtr, Xte = X[train], X[test]
    ytr, yte = y[train], y[test]
    members: List[Member] = []

    # ---------------------------------------------------------------- SVM x4
    svm_cfg = [("svm1", "linear", None), ("svm2", "linear", 0.5),
               ("svm3", "radial", None), ("svm4", "radial", 0.5)]
    for name, kern, wf in svm_cfg:
        def f(kern=kern, wf=wf):
            r = run_svm(50, kern, Xtr, ytr, Xte, yte, wf, genes)
            w = r["weightsvect"]
            return {"values": None if w is None else w.cpu().numpy(),
                    "metrics": r["test_metrics"], "options": r["options_string"][:1]}
        members.append((f"{name}_weights", f))

    # ---------------------------------------------------------------- lasso reps (one member)
    def lasso_member():
        reps = iterative_exclusion(X, y, genes, train, test, reps=lasso_reps, seed=seed)
        return {"reps": [{"nonzero_coef": r["nonzero_coef"], "metrics": r["test_metrics"],
                          "test_error": r["test_error"], "lambda_min": r["cv_fit"]["lambda_min"]}
                         for r in reps]}
    members.append(("lasso", lasso_member))

    # ---------------------------------------------------------------- random forests
    for nt in rf_trees:
        def f(nt=nt):
            rf = HistForest(nt, max_depth=10, seed=seed).fit(Xtr, ytr)
            pred = rf.predict(Xte).cpu()
            return {"values": rf.mean_decrease_gini.numpy(),
                    "metrics": binary_metrics(yte.cpu(), pred)}
        members.append((f"rfnb_{nt}_MeanDecGini", f))

    # ---------------------------------------------------------------- boosted trees
    for i, cfg in enumerate(xgb_configs):
        def f(cfg=cfg):
            m = HistBoost(cfg.get("n_estimators", 50), cfg.get("eta", 1.0),
                                     cfg.get("max_depth", 6), seed=seed).fit(Xtr, ytr)
            pred = (m.predict_proba(Xte)[:, 1] > 0.5).long().cpu()
            return {"values": m.feature_importances_.numpy(),
                    "metrics": binary_metrics(yte.cpu(), pred)}
        members.append((f"xg{i + 1}_imp", f))

    results = _run_members(members)

    # ---------------------------------------------------------------- assemble the table
    perf = {}
    for name, r in results.items():
        if name == "lasso":
            for k, rep in enumerate(r["reps"]):
                table.add(f"lasso_coef_rep{k + 1}", rep["nonzero_coef"])
                perf[f"lasso_rep{k + 1}"] = rep["metrics"]
            continue
        if r["values"] is None:
            table.df[name] = np.nan
        else:
            table.add(name, r["values"])
        perf[name] = r["metrics"]
    runs = [c for c in table.runs]
    table.add_consensus(runs, trim=1)
    sets = {c: selected(table.df[c]) for c in runs}
    out = {"table": table, "deg": deg, "performance": pd.DataFrame(perf).T,
           "intersections": {k: sorted(v) for k, v in intersections(
               {k: sets[k] for k in runs[:3]}).items()},
           "membership": membership_table(sets), "genes": genes,
           "train_idx": train.tolist(), "test_idx": test.tolist()}
    if out_dir and (not dist.is_initialized() or dist.get_rank() == 0):
        os.makedirs(out_dir, exist_ok=True)
        table.to_csv(os.path.join(out_dir, "standouttable.csv"))
        deg.to_csv(os.path.join(out_dir, "deg_table.csv"))
        out["performance"].to_csv(os.path.join(out_dir, "model_performance.csv"))
        out["membership"].to_csv(os.path.join(out_dir, "membership.csv"))
        with open(os.path.join(out_dir, "summary.json"), "w") as fh:
            json.dump({"n_genes": len(genes), "runs": runs,
                       "consensus_all_models": int((table.df["consensus_votes"] == len(runs)).sum()),
                       "intersections": {k: len(v) for k, v in out["intersections"].items()}},
                      fh, indent=1)
    return out
