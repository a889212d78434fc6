"""Ingestion, sample filtering and the expression container (reference layers L0-L5).

Re-designs of the reference's data plumbing (no network here, so GDC download C01 and biomaRt
annotation C09 take local files):

* ``concat_count_files``      C02 ``catExpnData`` (`JSmith_code/Cat_Expn_Data.r:7-49`)
* ``merge_manifest_clinical`` C03 (`scripts/clean.py:1-18`)
* ``transpose_assay``         C04 (`scripts/clean.py:21-41`)
* ``merge_assay_clinical``    C05 (`scripts/clean.py:43-72`)
* ``one_hot_like_train``      C06 (`scripts/dummies.py:1-29`, incl. its missing-import bug fixed)
* ``select_primary_samples``  C08 (`composite_code/rnotebook/seobjects/make_seobj_targetaml.R:55-78`)
* ``annotate_genes``          C09 from a local table (`make_seobj_targetaml.R:98-160`)
* ``ExpressionSet``           C10 SummarizedExperiment analogue (`make_seobj_targetaml.R:162-252`)
* ``synthetic_cohort``        TARGET-AML-shaped synthetic data (genes x samples counts, risk
                              labels, clinical table) for tests and benchmarks.
"""
from __future__ import annotations

import json
import os
import re
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np
import pandas as pd
import torch

USI_LEN = 16   # "TARGET-20-PANXXX" patient id prefix of entity_submitter_id


# ----------------------------------------------------------------------------- ingestion
def concat_count_files(paths: Sequence[str], names: Optional[Sequence[str]] = None,
                       gene_col: int = 0, value_col: int = 1, sep: str = "\t",
                       drop_special: bool = True) -> pd.DataFrame:
    """Column-bind per-sample count files (genes x samples). HTSeq's trailing ``__*`` summary
    rows are dropped when ``drop_special``. Gene order must agree across files."""
    cols = {}
    genes = None
    for i, p in enumerate(paths):
        df = pd.read_csv(p, sep=sep, header=None, comment=None)
        g = df.iloc[:, gene_col].astype(str)
        v = df.iloc[:, value_col]
        if drop_special:
            keep = ~g.str.startswith("__")
            g, v = g[keep], v[keep]
        if genes is None:
            genes = g.tolist()
        elif genes != g.tolist():
            raise ValueError(f"gene order of {p} differs from the first file")
        name = names[i] if names is not None else os.path.basename(p).split(".")[0]
        cols[name] = v.to_numpy()
    return pd.DataFrame(cols, index=genes)


def merge_manifest_clinical(manifest: pd.DataFrame, clinical: pd.DataFrame, project: str,
                            project_col: str = "project.project_id",
                            id_col: str = "entity_submitter_id",
                            usi_col: str = "TARGET USI") -> pd.DataFrame:
    m = manifest.loc[manifest[project_col] == project].copy()
    m[usi_col] = m[id_col].str.slice(0, USI_LEN)
    return clinical.merge(m, on=usi_col)


def transpose_assay(assay: pd.DataFrame, id_col: str = "entity_submitter_id",
                    gene_col_first: bool = True) -> pd.DataFrame:
    """genes x samples -> samples x genes, sample id kept as a column. When the first column
    holds gene ids (raw CSV) it becomes the header."""
    a = assay.set_index(assay.columns[0]) if gene_col_first and not np.issubdtype(
        assay.iloc[:, 0].dtype, np.number) else assay
    t = a.T.copy()
    t.columns = [str(c) for c in t.columns]
    t[id_col] = t.index.astype(str)
    return t


def merge_assay_clinical(assay_t: pd.DataFrame, clinical: pd.DataFrame,
                         id_col: str = "entity_submitter_id") -> pd.DataFrame:
    """Left-join clinical rows with assay rows on sample id (``-`` normalised to ``.``), add
    ``Diagnostic ID`` (tissue code, e.g. 03A/09A) as the second column."""
    c = clinical.copy()
    c[id_col] = c[id_col].astype(str).str.replace("-", ".", regex=False)
    out = c.merge(assay_t, how="left", on=id_col)
    out["Diagnostic ID"] = out[id_col].str.slice(-7, -4)
    cols = list(out.columns)
    order = [cols[0], "Diagnostic ID"] + [k for k in cols[1:] if k != "Diagnostic ID"]
    return out[order]


def one_hot_like_train(test_col: pd.Series, train_values: Iterable, name: str) -> pd.DataFrame:
    """One-hot columns for the *training* vocabulary; unseen test values map to all zeros."""
    return pd.DataFrame({f"{name}_{v}": (test_col == v).astype(int) for v in train_values},
                        index=test_col.index)


def one_hot_frame(df: pd.DataFrame, categories: Sequence[str]) -> pd.DataFrame:
    parts = [df] + [one_hot_like_train(df[c], df[c].unique(), c) for c in categories]
    return pd.concat(parts, axis=1)


def select_primary_samples(ids: Sequence[str], tissue_codes=("03A", "09A"),
                           project_code: str = ".20.") -> List[int]:
    """Indices of primary diagnostic samples (tissue code in ``tissue_codes``) of one project,
    matching ``TARGET.20.PAXXXX.09A.01R``-style ids (either ``-`` or ``.`` separators)."""
    keep = []
    for i, s in enumerate(ids):
        t = str(s).replace("-", ".")
        if project_code in t and any(f".{c}." in t or t.endswith(c) for c in tissue_codes):
            keep.append(i)
    return keep


def annotate_genes(gene_ids: Sequence[str], table: pd.DataFrame,
                   key: str = "ensembl_gene_id") -> pd.DataFrame:
    """Join versioned Ensembl ids (``ENSG...15``) with a local annotation table."""
    base = [re.sub(r"\.\d+$", "", g) for g in gene_ids]
    ann = table.drop_duplicates(key).set_index(key)
    out = ann.reindex(base)
    out.index = list(gene_ids)
    out[key] = base
    return out


# ----------------------------------------------------------------------------- container
@dataclass
class ExpressionSet:
    """Genes x samples assays with row (gene) and column (sample) annotations.

    ``assays`` maps a name ("counts", "logcpm", ...) to a float tensor [genes, samples].
    """
    assays: Dict[str, torch.Tensor]
    genes: List[str]
    samples: List[str]
    row_data: pd.DataFrame = field(default_factory=pd.DataFrame)
    col_data: pd.DataFrame = field(default_factory=pd.DataFrame)

    def __post_init__(self):
        for k, v in self.assays.items():
            if tuple(v.shape) != (len(self.genes), len(self.samples)):
                raise ValueError(f"assay {k} has shape {tuple(v.shape)}, expected "
                                 f"{(len(self.genes), len(self.samples))}")

    @property
    def shape(self):
        return len(self.genes), len(self.samples)

    def subset(self, genes=None, samples=None) -> "ExpressionSet":
        gi = _index(genes, self.genes)
        si = _index(samples, self.samples)
        assays = {k: v[gi][:, si] for k, v in self.assays.items()}
        rd = self.row_data.iloc[gi] if len(self.row_data) else self.row_data
        cd = self.col_data.iloc[si] if len(self.col_data) else self.col_data
        return ExpressionSet(assays, [self.genes[i] for i in gi], [self.samples[i] for i in si],
                             rd, cd)

    def to(self, device) -> "ExpressionSet":
        return ExpressionSet({k: v.to(device) for k, v in self.assays.items()}, self.genes,
                             self.samples, self.row_data, self.col_data)

    def save(self, path: str) -> None:
        """Directory with assays.safetensors + genes/samples/row/col tables (no pickle)."""
        from safetensors.torch import save_file
        os.makedirs(path, exist_ok=True)
        save_file({k: v.contiguous().cpu() for k, v in self.assays.items()},
                  os.path.join(path, "assays.safetensors"))
        with open(os.path.join(path, "meta.json"), "w") as fh:
            json.dump({"genes": self.genes, "samples": self.samples}, fh)
        self.row_data.to_csv(os.path.join(path, "row_data.csv"))
        self.col_data.to_csv(os.path.join(path, "col_data.csv"))

    @classmethod
    def from_rdata(cls, path: str, name: Optional[str] = None,
                   assay_name: str = "logcpm") -> "ExpressionSet":
        """A SummarizedExperiment saved by the reference (e.g.
        ``composite_code/rnotebook/data/sesetfilt_degseahack_targetaml.rda``, the 1984 x 137 DEG
        container loaded at `cml_targetaml_seanalysis.Rmd:409-415`), through the data-only reader
        ``select.rdata``. The first assay is stored as ``assay_name`` (the reference's analysis
        assay is TMM log-CPM); row_data holds the DE statistics of its rowRanges."""
        from .rdata import read_rdata, summarized_experiment
        objs = read_rdata(path)
        obj = objs[name] if name else next(iter(objs.values()))
        se = summarized_experiment(obj)
        assays = {}
        for i, (k, v) in enumerate(se["assays"].items()):
            assays[assay_name if i == 0 else k] = torch.as_tensor(v, dtype=torch.float32)
        return cls(assays, list(se["genes"]), list(se["samples"]), se["row_data"], se["col_data"])

    @classmethod
    def load(cls, path: str) -> "ExpressionSet":
        from safetensors.torch import load_file
        assays = load_file(os.path.join(path, "assays.safetensors"))
        with open(os.path.join(path, "meta.json")) as fh:
            meta = json.load(fh)
        rd = pd.read_csv(os.path.join(path, "row_data.csv"), index_col=0)
        cd = pd.read_csv(os.path.join(path, "col_data.csv"), index_col=0)
        return cls(dict(assays), meta["genes"], meta["samples"], rd, cd)


def _index(sel, names: List[str]) -> List[int]:
    if sel is None:
        return list(range(len(names)))
    if isinstance(sel, torch.Tensor):
        sel = sel.tolist()
    sel = list(sel)
    if sel and isinstance(sel[0], bool):
        return [i for i, b in enumerate(sel) if b]
    if sel and isinstance(sel[0], str):
        pos = {n: i for i, n in enumerate(names)}
        return [pos[s] for s in sel]
    return [int(i) for i in sel]


# ----------------------------------------------------------------------------- synthetic data
def synthetic_cohort(n_genes: int = 2000, n_samples: int = 145, n_signal: int = 40,
                     effect: float = 1.5, seed: int = 2019, depth: float = 2e7) -> ExpressionSet:
    """TARGET-AML-shaped synthetic RNA-seq: negative-binomial counts, a binary risk label
    (``low_risk``: 1 = Low, 0 = Standard/High) driven by ``n_signal`` genes, library-size
    variation, and a 2/3 train split flag (``exptset``), as in `make_seobj_targetaml.R:81-82`."""
    g = np.random.default_rng(seed)
    base = g.lognormal(mean=3.0, sigma=2.0, size=n_genes)
    base = base / base.sum()
    y = (g.random(n_samples) < 0.45).astype(np.int64)
    lfc = np.zeros(n_genes)
    sig = g.choice(n_genes, n_signal, replace=False)
    lfc[sig] = g.choice([-1, 1], n_signal) * effect * (0.5 + g.random(n_signal))
    lib = depth * g.lognormal(0, 0.3, size=n_samples)
    mu = base[:, None] * lib[None, :] * np.exp(lfc[:, None] * y[None, :])
    disp = 0.1
    lam = g.gamma(1 / disp, mu * disp)
    counts = g.poisson(lam).astype(np.float32)
    genes = [f"ENSG{100000 + i:011d}.{1 + i % 9}" for i in range(n_genes)]
    samples = [f"TARGET.20.PA{i:04d}.09A.01R" for i in range(n_samples)]
    train = np.zeros(n_samples, dtype=bool)
    train[g.permutation(n_samples)[: int(round(2 * n_samples / 3))]] = True
    col = pd.DataFrame({"low_risk": y, "exptset": np.where(train, "train", "test"),
                        "age": g.integers(1, 20, n_samples),
                        "gender": g.choice(["Male", "Female"], n_samples)}, index=samples)
    row = pd.DataFrame({"true_lfc": lfc, "signal": np.isin(np.arange(n_genes), sig)},
                       index=genes)
    return ExpressionSet({"counts": torch.from_numpy(counts)}, genes, samples, row, col)


def target_aml_cohort(clinical_csv: str, train_csv: str, test_csv: str) -> pd.DataFrame:
    """The reference's TARGET-AML analysis cohort from its own files (C08/C12/C30).

    Patients of the seeded 2/3 split (``JSmith_code/TARGET_AML_{Training,Testing}_Samples.csv``,
    `Differential_Expression_and_Lasso.Rmd:158-187`) joined to the clinical table
    (``Clinical_Data/AML_dataframe.csv``), first occurrence per USI (`scripts/README.md:6`), with
    the reference's binarised risk label ``deg_risk`` (Low = 0; Standard / High = 1; Unknown =
    NA, `cml_targetaml_seanalysis.Rmd:435-436`) and ``exptset`` = train | test
    (`make_seobj_targetaml.R:81-82`). Columns are renamed to snake case: gender, age_days,
    risk_group."""
    clin = pd.read_csv(clinical_csv)
    train = pd.read_csv(train_csv)["x"].tolist()
    test = pd.read_csv(test_csv)["x"].tolist()
    split = {u: "train" for u in train}
    split.update({u: "test" for u in test})
    sub = clin[clin["TARGET USI"].isin(split)].drop_duplicates("TARGET USI")
    out = pd.DataFrame({
        "usi": sub["TARGET USI"].values,
        "gender": sub["Gender"].values,
        "age_days": sub["Age at Diagnosis in Days"].values,
        "risk_group": sub["Risk group"].values,
    })
    out["deg_risk"] = out["risk_group"].map({"Low": 0, "Standard": 1, "High": 1})
    out["exptset"] = out["usi"].map(split)
    return out.set_index("usi")
