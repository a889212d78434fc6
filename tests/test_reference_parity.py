"""Parity with numbers the reference itself records, computed from the reference's own files
(read-only, /root/reference): the TARGET-AML cohort tables and chi-square balance tests of
`composite_code/rnotebook/cml_targetaml_seanalysis.Rmd:422-474` (golden values pasted there as
comments: risk-group counts, 137 samples after filtering, gender / age tables, p = 0.8044 and
p = 0.6591), and the column schema of the reference's standard output table."""
import os

import numpy as np
import pandas as pd
import pytest

REF = "/root/reference"
CLIN = os.path.join(REF, "Clinical_Data", "AML_dataframe.csv")
TRAIN = os.path.join(REF, "JSmith_code", "TARGET_AML_Training_Samples.csv")
TEST = os.path.join(REF, "JSmith_code", "TARGET_AML_Testing_Samples.csv")
STAND = os.path.join(REF, "composite_code", "rnotebook", "data", "standouttable.csv")

pytestmark = pytest.mark.skipif(not os.path.exists(CLIN), reason="reference files not present")


def test_target_aml_cohort_tables_and_chisq():
    from consensusml_amd.select.data import target_aml_cohort
    from consensusml_amd.select.stats import chisq_test, cohort_summary
    co = target_aml_cohort(CLIN, TRAIN, TEST)
    # SEA:428-433: dim 1984 x 145; High 8, Low 60, Standard 69, Unknown 8
    assert len(co) == 145
    assert co["risk_group"].value_counts().to_dict() == {"Standard": 69, "Low": 60, "Unknown": 8,
                                                        "High": 8}
    f = co[co["deg_risk"].notna()].copy()
    f["deg_risk"] = f["deg_risk"].astype(int)
    assert len(f) == 137                                    # SEA:454
    gt = pd.crosstab(f["gender"], f["deg_risk"])
    assert gt.loc["Female"].tolist() == [29, 40] and gt.loc["Male"].tolist() == [31, 37]
    p_gender = chisq_test(gt.to_numpy())["p_value"]
    assert round(p_gender, 4) == 0.8044                     # SEA:462
    summ = cohort_summary(f, label="deg_risk", covariates=("gender", "age_days"))
    assert round(summ["gender"]["p_value"], 4) == 0.8044
    age = summ["age_days"]
    tab = pd.DataFrame(age["table"])                        # rows: >= median (old) / < median
    old = [k for k in tab.index if k.startswith(">=")][0]
    young = [k for k in tab.index if k.startswith("<")][0]
    assert tab.loc[old].tolist() == [32, 37] and tab.loc[young].tolist() == [28, 40]   # SEA:466-467
    assert round(age["p_value"], 4) == 0.6591               # SEA:469
    # the split itself: 96 training / 49 testing patients (DEL:159-177)
    assert (co["exptset"] == "train").sum() == 96 and (co["exptset"] == "test").sum() == 49


def test_standard_table_schema_matches_reference(tmp_path):
    """Our StandardTable writes the reference's column layout: the DE statistics columns of
    rowData(deg.seset) followed by one column per model run (standouttable.csv:1)."""
    from consensusml_amd.select.consensus import StandardTable
    ref = pd.read_csv(STAND, nrows=5)
    de_cols = ["hgnc_id", "hgnc_symbol", "ensembl_gene_id", "logFC", "AveExpr", "t", "p.unadj",
               "p.adj.bh", "b"]
    assert list(ref.columns[1:10]) == de_cols
    genes = [f"ENSG{i:011d}" for i in range(6)]
    de = pd.DataFrame({c: np.arange(6, dtype=float) for c in de_cols[3:]}, index=genes)
    for c in de_cols[:3]:
        de[c] = [f"{c}{i}" for i in range(6)]
    t = StandardTable(genes, de[de_cols])
    model_cols = list(ref.columns[10:])
    for c in model_cols:
        t.add(c, np.linspace(0, 1, 6))
    assert list(t.df.columns) == de_cols + model_cols
    out = tmp_path / "standouttable.csv"
    t.to_csv(str(out))
    with open(STAND) as fh:
        ref_header = fh.readline().strip()
    with open(out) as fh:
        our_header = fh.readline().strip()
    assert our_header == ref_header                          # write.csv layout, same columns
    back = StandardTable.read_csv(str(out))
    assert list(back.df.columns) == de_cols + model_cols and back.genes == genes
