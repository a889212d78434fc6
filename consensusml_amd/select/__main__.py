"""Command line for the feature-selection consensus pipeline (the reference's notebook run,
`composite_code/rnotebook/cml_targetaml_seanalysis.Rmd`, as one command).

  # the reference's own analysis input: the DEG SummarizedExperiment it saved (1984 x 137
  # log-CPM; read by the data-only R reader) with its train/test split and risk labels —
  # the full reference run (4 SVMs, 15 lasso reps, RF 2k/5k/10k, 5 XGB configs) by default
  python -m consensusml_amd.select \
      --rdata composite_code/rnotebook/data/sesetfilt_degseahack_targetaml.rda --out out/
  # ... interrupted? continue from the last finished stage
  python -m consensusml_amd.select --rdata ... --out out/ --resume

  # TARGET-AML-shaped synthetic cohort (no data offline)
  python -m consensusml_amd.select --synthetic --out out/

  # real data: genes x samples count matrix (first column = gene id, as written by catExpnData),
  # the reference's clinical table and its seeded split files
  python -m consensusml_amd.select --counts counts.csv \\
      --clinical Clinical_Data/AML_dataframe.csv \\
      --train-ids JSmith_code/TARGET_AML_Training_Samples.csv \\
      --test-ids JSmith_code/TARGET_AML_Testing_Samples.csv --out out/

  # ensemble members sharded over ranks (importance vectors all-gathered)
  torchrun --nproc-per-node 4 --master-addr 127.0.0.1 -m consensusml_amd.select --synthetic

Count columns are matched to patients by their TARGET USI prefix (first 16 characters of the
sample id, `scripts/clean.py:1-18`). Output in ``--out``: ``standouttable.csv`` (reference
24-column layout), ``standouttable_extended.csv``, ``results/<family>_resultslist`` per stage
(JSON + safetensors), the incrementally saved ``standardtable_mloutputs_summary.csv`` and a JSON
summary.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import pandas as pd
import torch


def _load_counts(args):
    from .data import USI_LEN, ExpressionSet, target_aml_cohort
    counts = pd.read_csv(args.counts, index_col=0)
    cohort = target_aml_cohort(args.clinical, args.train_ids, args.test_ids)
    cohort = cohort[cohort["deg_risk"].notna()]
    cols = [c for c in counts.columns if c[:USI_LEN].replace(".", "-") in cohort.index]
    usi = [c[:USI_LEN].replace(".", "-") for c in cols]
    col = cohort.loc[usi].reset_index()
    col.index = cols
    # the pipeline's label: 1 = Low risk (the reference binarises Low = 0 vs Standard/High = 1;
    # either coding gives the same selections)
    col["low_risk"] = (col["deg_risk"] == 0).astype(int)
    X = torch.as_tensor(counts[cols].to_numpy(dtype="float64"), dtype=torch.float32)
    return ExpressionSet({"counts": X}, [str(g) for g in counts.index], cols, col_data=col)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    src = ap.add_mutually_exclusive_group(required=True)
    src.add_argument("--synthetic", action="store_true", help="TARGET-AML-shaped synthetic cohort")
    src.add_argument("--counts", help="genes x samples raw count CSV")
    src.add_argument("--rdata", help="the reference's DEG SummarizedExperiment (.rda)")
    ap.add_argument("--label-col", default=None, help="label column (default: deg.risk for "
                    "--rdata, low_risk otherwise)")
    ap.add_argument("--split-col", default=None, help="train/test column (default: "
                    "exptset.seahack for --rdata, exptset otherwise)")
    ap.add_argument("--resume", action="store_true", help="skip stages whose results exist")
    ap.add_argument("--tree-method", choices=["exact", "hist"], default="exact")
    ap.add_argument("--xgb-configs", default=None,
                    help='JSON list of {"max_depth", "n_estimators"} (default: the reference 5)')
    ap.add_argument("--no-proximity", action="store_true", help="skip RF proximity matrices")
    ap.add_argument("--clinical", help="clinical CSV (Clinical_Data/AML_dataframe.csv layout)")
    ap.add_argument("--train-ids", help="training USIs CSV (reference split file)")
    ap.add_argument("--test-ids", help="testing USIs CSV (reference split file)")
    ap.add_argument("--genes", type=int, default=2000, help="synthetic: number of genes")
    ap.add_argument("--samples", type=int, default=145, help="synthetic: number of samples")
    ap.add_argument("--max-genes", type=int, default=None, help="cap on DE genes carried forward")
    ap.add_argument("--lasso-reps", type=int, default=15)
    ap.add_argument("--rf-trees", type=int, nargs="+", default=[2000, 5000, 10000])
    ap.add_argument("--seed", type=int, default=2019)
    ap.add_argument("--device", default="auto", help="cuda | cpu | auto")
    ap.add_argument("--out", default="consensus_out")
    a = ap.parse_args(argv)
    from .data import synthetic_cohort
    from .pipeline import consensus_pipeline
    if a.counts and not (a.clinical and a.train_ids and a.test_ids):
        ap.error("--counts needs --clinical, --train-ids and --test-ids")
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        from ..parallel.dist import init_distributed
        init_distributed("gloo" if a.device == "cpu" else "auto")
    dev = torch.device("cuda" if (a.device == "auto" and torch.cuda.is_available())
                       else ("cpu" if a.device == "auto" else a.device))
    from .pipeline import REF_XGB
    xgb = tuple(json.loads(a.xgb_configs)) if a.xgb_configs else REF_XGB
    kw = dict(out_dir=a.out, seed=a.seed, lasso_reps=a.lasso_reps, rf_trees=tuple(a.rf_trees),
              device=dev, max_genes=a.max_genes, xgb_configs=xgb, resume=a.resume,
              tree_method=a.tree_method, rf_proximity=not a.no_proximity)
    if a.rdata:
        from .data import ExpressionSet
        es = ExpressionSet.from_rdata(a.rdata)
        res = consensus_pipeline(es, label_col=a.label_col or "deg.risk",
                                 split_col=a.split_col or "exptset.seahack",
                                 deg_from_container=True, **kw)
    else:
        es = synthetic_cohort(a.genes, a.samples, seed=a.seed) if a.synthetic else _load_counts(a)
        res = consensus_pipeline(es, label_col=a.label_col or "low_risk",
                                 split_col=a.split_col or "exptset", **kw)
    inter = res.get("intersections", {})
    print(json.dumps({"out": a.out, "samples": len(es.samples), "genes": len(es.genes),
                      "resumed_stages": res.get("resumed_stages", []),
                      "intersection_sizes": {k: len(v) for k, v in inter.items()}}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
