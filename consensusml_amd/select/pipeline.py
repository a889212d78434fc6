"""End-to-end feature-selection consensus pipeline (reference call stack SURVEY.md §3.2 / §3.3).

``consensus_pipeline`` mirrors `composite_code/rnotebook/cml_targetaml_seanalysis.Rmd` end to end:
(DE genes on the training split, or the reference's DEG container as is) -> standard table
seeded with the DE statistics -> 4 SVM runs (linear / radial x 50 % weight filter, `:647-667`)
-> 15 iterative-exclusion lasso reps (`:728-776`) -> random forests with 2k / 5k / 10k trees and
proximity (`:1037-1050`) -> the 5 XGBoost configurations (`:1164-1186`) -> consensus columns.
Those are the defaults; smaller runs pass smaller settings.

Persistence and resume follow the reference's stage pattern (`:672-690`, `:778-799`,
`:1069-1091`, `:1239-1263`): after each stage its named result list is saved
(``results/<name>`` via ``select.results``: JSON + safetensors, never pickle) and the standard
table is re-written with the stage's columns appended (``standardtable_mloutputs_summary.csv``).
With ``resume=True`` a stage whose result list exists is not recomputed: its columns are taken
from the saved table, so an interrupted run continues where it stopped.

Outputs: ``standouttable.csv`` in the reference's 24-column layout (DE statistics, lasso reps
1-3, rfnb_{2k,5k,10k}, svm1-4, xg1-5), ``standouttable_extended.csv`` (every rep + consensus
columns), model performance, membership table and a JSON summary.

Defects of the reference are not reproduced (§4.3): every rep's coefficients are kept, SVM
weights come from the refit model, XGB metrics use each model's own predictions.

Ensemble parallelism: within a stage the model runs ("members") are independent, so with a
process group each rank runs members[rank::world] and the results are all-gathered — the same
"workers as ranks" structure as the data-parallel engine.
"""
from __future__ import annotations

import json
import time
import os
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import pandas as pd
import torch
import torch.distributed as dist

from . import results as RS
from .consensus import StandardTable, intersections, membership_table, selected
from .data import ExpressionSet
from .de import voom_de
from .lasso import iterative_exclusion
from .metrics import binary_metrics, confusion_matrix
from .normalize import normalize
from .svm import run_svm

Member = Tuple[str, Callable[[], Dict[str, object]]]

# the reference's model runs
REF_SVM = (("svm1", "linear", None), ("svm2", "linear", 0.5), ("svm3", "radial", None),
           ("svm4", "radial", 0.5))                                           # SEA:647-667
REF_LASSO_REPS = 15                                                          # SEA:728-776
REF_RF_TREES = (2000, 5000, 10000)                                           # SEA:1037-1050
REF_XGB = ({"max_depth": 2, "n_estimators": 2}, {"max_depth": 50, "n_estimators": 2},
           {"max_depth": 50, "n_estimators": 50}, {"max_depth": 100, "n_estimators": 50},
           {"max_depth": 100, "n_estimators": 100})                          # SEA:1164-1186
DE_COLUMNS = ["hgnc_id", "hgnc_symbol", "ensembl_gene_id", "logFC", "AveExpr", "t", "p.unadj",
              "p.adj.bh", "b"]
TABLE_FILE = "standardtable_mloutputs_summary.csv"


def rf_column(ntree: int) -> str:
    return f"rfnb_{ntree // 1000}k_MeanDecNodeImp" if ntree % 1000 == 0 else \
        f"rfnb_{ntree}_MeanDecNodeImp"


def _run_members(members: List[Member]) -> Dict[str, Dict[str, object]]:
    """Run members (sharded over ranks when a process group exists) and gather their results
    on every rank."""
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


def _is_writer() -> bool:
    return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0


class _Stages:
    """Stage bookkeeping: result lists + the incrementally saved standard table."""

    def __init__(self, out_dir: Optional[str], resume: bool, table: StandardTable):
        self.out_dir, self.resume, self.table = out_dir, resume and out_dir is not None, table
        self.saved = None
        if self.resume and os.path.exists(self._p(TABLE_FILE)):
            self.saved = pd.read_csv(self._p(TABLE_FILE), index_col=0)
        self.skipped: List[str] = []

    def _p(self, *parts) -> str:
        return os.path.join(self.out_dir, *parts)

    def done(self, name: str, columns: Sequence[str] = ()) -> bool:
        """A stage is finished when its result list (the commit marker, written last) exists
        and the saved table holds every column the stage would add now (a run with other
        lasso_reps / svm_runs / tree counts re-runs the stage instead of failing in restore)."""
        return (self.resume and self.saved is not None and RS.exists(self._p("results", name))
                and all(c in self.saved.columns for c in columns))

    def restore(self, name: str, columns: Sequence[str]) -> Dict[str, object]:
        """Reload a finished stage: its result list and its table columns."""
        for c in columns:
            self.table.df[c] = self.saved.loc[self.table.genes, c].to_numpy()
            self.table.runs.append(c)
        self.skipped.append(name)
        return RS.load_results(self._p("results", name))

    def finish(self, name: str, resultslist: Dict[str, object]) -> None:
        if self.out_dir is None or not _is_writer():
            return
        # the table first, the result list last: the result list is the stage's commit marker
        # (done()), so an interruption between the two writes re-runs the stage
        os.makedirs(self.out_dir, exist_ok=True)
        tmp = self._p(TABLE_FILE + ".part")
        self.table.df.to_csv(tmp)
        os.replace(tmp, self._p(TABLE_FILE))
        RS.save_results(self._p("results", name), resultslist)


def consensus_pipeline(es: ExpressionSet, label_col: str = "low_risk",
                       split_col: str = "exptset", out_dir: Optional[str] = None,
                       seed: int = 2019, lasso_reps: int = REF_LASSO_REPS,
                       rf_trees: Sequence[int] = REF_RF_TREES, rf_proximity: bool = True,
                       xgb_configs: Sequence[dict] = REF_XGB, svm_runs=REF_SVM,
                       de_lfc: float = 1.0, device: Optional[torch.device] = None,
                       max_genes: Optional[int] = None, deg_from_container: bool = False,
                       tree_method: str = "exact", resume: bool = False) -> Dict[str, object]:
    """Run the reference analysis. ``deg_from_container``: ``es`` is already the DEG container
    (the reference starts from ``sesetfilt_degseahack_targetaml.rda``: log-CPM of 1984 DEGs with
    the DE statistics in row_data), so no DE step. ``tree_method``: "exact" (CART / exact greedy
    boosting, the reference's randomForest / xgboost semantics) or "hist" (histogram trees with
    the HIP split kernels, for large problems on the GPU)."""
    dev = device or torch.device("cpu")
    y_all = torch.as_tensor(pd.to_numeric(es.col_data[label_col]).to_numpy(), dtype=torch.long)
    split = es.col_data[split_col].astype(str).to_numpy()
    train = np.where(split == "train")[0]
    test = np.where(split == "test")[0]

    # ---------------------------------------------------------------- DE genes / container
    if deg_from_container:
        genes = list(es.genes)
        deg = es.row_data.copy()
        X_all = es.assays["logcpm"]
    else:
        if "logcpm" not in es.assays:
            es = normalize(es)
        cnt = es.assays["counts"]
        deg = voom_de(cnt[:, train], y_all[train].tolist(), es.genes, lfc=de_lfc)
        deg = deg.rename(columns={"P.Value": "p.unadj", "adj.P.Val": "p.adj.bh", "B": "b"})
        genes = list(deg.index)
        X_all = None
    if max_genes is not None:
        genes = genes[:max_genes]
    if len(genes) < 2:
        raise RuntimeError("fewer than 2 differentially expressed genes")
    sub = es.subset(genes=genes)
    X = sub.assays["logcpm"].t().contiguous().float().to(dev)          # samples x genes
    y = y_all.to(dev)
    base = deg.loc[genes]
    base = base[[c for c in DE_COLUMNS if c in base.columns] +
                [c for c in base.columns if c not in DE_COLUMNS]]
    table = StandardTable(genes, base)
    st = _Stages(out_dir, resume, table)
    Xtr, Xte = X[train], X[test]
    ytr, yte = y[train], y[test]
    perf: Dict[str, dict] = {}
    stage_s: Dict[str, float] = {}     # wall seconds per stage (device-synchronised)
    clock = [time.perf_counter()]

    def lap(name: str) -> None:
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        now = time.perf_counter()
        stage_s[name] = round(now - clock[0], 3)
        clock[0] = now

    # ---------------------------------------------------------------- SVM (svm4reps)
    svm_cols = [f"{n}_weights" for n, _, _ in svm_runs]
    if st.done("svm4reps_resultslist", svm_cols):
        svm_res = st.restore("svm4reps_resultslist", svm_cols)
    else:
        members: List[Member] = []
        for name, kern, wf in svm_runs:
            def f(kern=kern, wf=wf):
                r = run_svm(50, kern, Xtr, ytr, Xte, yte, wf, genes)
                w = r["weightsvect"]
                return {"options_string": r["options_string"][:1],
                        "weightsvect": None if w is None else w.cpu().numpy(),
                        "features_used": len(r["features_used"]),
                        "predictions_train": r["predictions_train"].numpy(),
                        "predictions_test": r["predictions_test"].numpy(),
                        "decision_values_test": r["decision_values_test"].numpy(),
                        "performance_test": {k: np.asarray(v) for k, v in
                                             r["performance_test"].items()},
                        "TPR_test": r["TPR_test"], "precision_test": r["precision_test"],
                        "recall_test": r["recall_test"], "test_metrics": r["test_metrics"]}
            members.append((name, f))
        svm_res = _run_members(members)
        for (name, _, _), col in zip(svm_runs, svm_cols):
            w = svm_res[name]["weightsvect"]
            if w is None:
                table.df[col] = np.nan
                table.runs.append(col)
            else:
                table.add(col, w)
        st.finish("svm4reps_resultslist", svm_res)
    for name, _, _ in svm_runs:
        perf[f"{name}_weights"] = svm_res[name]["test_metrics"]
    lap("svm")

    # ---------------------------------------------------------------- lasso reps
    lasso_cols = [f"lasso_coef_rep{k + 1}" for k in range(lasso_reps)]
    if st.done("lasso_resultslist", lasso_cols):
        lasso_res = st.restore("lasso_resultslist", lasso_cols)
    else:
        def lasso_member():
            reps = iterative_exclusion(X, y, genes, train, test, reps=lasso_reps, seed=seed)
            out = {}
            for r in reps:
                cv = r["cv_fit"]
                out[f"rep{r['rep']}"] = {
                    "training.set": [es.samples[i] for i in r["training_set"]],
                    "testing.set": [es.samples[i] for i in r["testing_set"]],
                    "contrast": r["contrast"],
                    "cv.fit": {"lambda": cv["lambda"], "cvm": cv["cvm"], "cvsd": cv["cvsd"],
                               "lambda.min": cv["lambda_min"], "lambda.1se": cv["lambda_1se"]},
                    "confusionMatrix": r["confusion_matrix"].numpy(),
                    "test.error": r["test_error"], "nonzero.coef": r["nonzero_coef"],
                    "excluded_before": len(r["excluded_before"]), "seed": r["seed"],
                    "test_metrics": r["test_metrics"]}
            return out
        lasso_res = _run_members([("lasso", lasso_member)])["lasso"]
        for k in range(lasso_reps):
            rep = lasso_res.get(f"rep{k + 1}")
            table.add(lasso_cols[k], rep["nonzero.coef"] if rep else {})
        st.finish("lasso_resultslist", lasso_res)
    for k in range(lasso_reps):
        rep = lasso_res.get(f"rep{k + 1}")
        if rep:
            perf[f"lasso_rep{k + 1}"] = rep["test_metrics"]
    lap("lasso")

    # ---------------------------------------------------------------- random forests
    rf_cols = [rf_column(n) for n in rf_trees]
    if st.done("rf_noboost_resultslist", rf_cols):
        rf_res = st.restore("rf_noboost_resultslist", rf_cols)
    else:
        members = []
        for nt in rf_trees:
            def f(nt=nt):
                if tree_method == "hist":
                    from .hist_trees import HistForest
                    rf = HistForest(nt, max_depth=10, seed=20).fit(Xtr, ytr)
                elif Xtr.is_cuda:
                    # exact thresholds, level-synchronous on the device (tree_hist.hip)
                    from .hist_trees import ExactForest
                    rf = ExactForest(nt, seed=20).fit(Xtr, ytr)
                else:
                    from .trees import RandomForest
                    rf = RandomForest(nt, seed=20).fit(Xtr, ytr)
                pred = rf.predict(Xte).cpu()
                out = {"importance": rf.mean_decrease_gini.numpy(),
                       "predicted_test": pred.numpy(),
                       "conf.matrix": confusion_matrix(yte.cpu(), pred, 2).numpy(),
                       "ntree": nt, "test_metrics": binary_metrics(yte.cpu(), pred),
                       # which split finder ran (ExactForest falls back to 128 quantile bins
                       # past 128 distinct training values per feature)
                       "split_method": {"exact": bool(getattr(rf, "exact", tree_method != "hist")),
                                        "bins": int(getattr(rf, "n_bins", 0) or 0),
                                        "impl": type(rf).__name__}}
                if rf_proximity:
                    out["proximity"] = rf.proximity(Xtr).cpu().numpy()
                return out
            members.append((f"rf{nt}", f))
        got = _run_members(members)
        rf_res = {f"rf{nt}.results": got[f"rf{nt}"] for nt in rf_trees}
        for nt, col in zip(rf_trees, rf_cols):
            table.add(col, rf_res[f"rf{nt}.results"]["importance"])
        st.finish("rf_noboost_resultslist", rf_res)
    for nt, col in zip(rf_trees, rf_cols):
        perf[col] = rf_res[f"rf{nt}.results"]["test_metrics"]
    lap("random_forest")

    # ---------------------------------------------------------------- boosted trees
    xgb_cols = [f"xg{i + 1}_imp" for i in range(len(xgb_configs))]
    if st.done("xgb_resultslist", xgb_cols):
        xgb_res = st.restore("xgb_resultslist", xgb_cols)
    else:
        members = []
        for i, cfg in enumerate(xgb_configs):
            def f(cfg=cfg):
                if tree_method == "hist":
                    from .hist_trees import HistBoost
                    m = HistBoost(cfg.get("n_estimators", 50), cfg.get("eta", 1.0),
                                  cfg.get("max_depth", 6), seed=seed).fit(Xtr, ytr)
                    imp = m.feature_importances_.numpy()
                else:
                    from .trees import GradientBoostedTrees
                    m = GradientBoostedTrees(cfg.get("n_estimators", 50), cfg.get("eta", 1.0),
                                             cfg.get("max_depth", 6)).fit(Xtr, ytr)
                    imp = m.importance.numpy()
                    imp = imp / imp.sum() if imp.sum() > 0 else imp
                prob = m.predict_proba(Xte)[:, 1].cpu()
                pred = (prob > 0.5).long()
                met = binary_metrics(yte.cpu(), pred)
                return {"importance": imp, "params": dict(cfg, eta=cfg.get("eta", 1.0),
                                                          objective="binary:logistic"),
                        "performance_testset": {
                            "confusionMatrix": confusion_matrix(yte.cpu(), pred, 2).numpy(),
                            "mean_err": float((pred != yte.cpu()).float().mean()),
                            "tpr": met["tpr"], "tnr": met["tnr"], "fdr": met["fdr"],
                            "for": met["for"]},
                        "test_metrics": met}
            members.append((f"rep{i + 1}", f))
        xgb_res = _run_members(members)
        xgb_res["testperfdf"] = {k: {m: v["performance_testset"][m]
                                     for m in ("mean_err", "tpr", "tnr", "fdr", "for")}
                                 for k, v in xgb_res.items()}
        for i, col in enumerate(xgb_cols):
            table.add(col, xgb_res[f"rep{i + 1}"]["importance"])
        st.finish("xgb_resultslist", xgb_res)
    for i, col in enumerate(xgb_cols):
        perf[col] = xgb_res[f"rep{i + 1}"]["test_metrics"]
    lap("boosted_trees")

    # ---------------------------------------------------------------- consensus
    runs = list(table.runs)
    valid = [c for c in runs if table.df[c].notna().all()]
    table.add_consensus(valid, trim=1)
    sets = {c: selected(table.df[c]) for c in valid}
    first3 = [c for c in (svm_cols[:1] + lasso_cols[:1] + rf_cols[:1] + xgb_cols[:1]) if c in sets]
    out = {"table": table, "deg": deg, "performance": pd.DataFrame(perf).T,
           "intersections": {k: sorted(v) for k, v in intersections(
               {k: sets[k] for k in first3[:3]}).items()},
           "membership": membership_table(sets), "genes": genes,
           "train_idx": train.tolist(), "test_idx": test.tolist(),
           "resultslists": {"svm": svm_res, "lasso": lasso_res, "rf": rf_res, "xgb": xgb_res},
           "resumed_stages": list(st.skipped), "stage_seconds": stage_s}
    if out_dir and _is_writer():
        os.makedirs(out_dir, exist_ok=True)
        ref_cols = [c for c in DE_COLUMNS if c in table.df.columns] + \
            lasso_cols[:3] + rf_cols + svm_cols + xgb_cols
        ref_table = StandardTable(genes, table.df[ref_cols])
        ref_table.to_csv(os.path.join(out_dir, "standouttable.csv"))
        table.to_csv(os.path.join(out_dir, "standouttable_extended.csv"))
        deg.to_csv(os.path.join(out_dir, "deg_table.csv"))
        out["performance"].to_csv(os.path.join(out_dir, "model_performance.csv"))
        out["membership"].to_csv(os.path.join(out_dir, "membership.csv"))
        with open(os.path.join(out_dir, "summary.json"), "w") as fh:
            json.dump({"n_genes": len(genes), "runs": runs, "resumed_stages": st.skipped,
                       "rf_split_method": {f"rf{nt}": rf_res[f"rf{nt}.results"].get("split_method")
                                           for nt in rf_trees},
                       "device": str(dev), "stage_seconds": stage_s,
                       "consensus_all_models": int((table.df["consensus_votes"] ==
                                                    len(valid)).sum()),
                       "intersections": {k: len(v) for k, v in out["intersections"].items()}},
                      fh, indent=1)
    return out
