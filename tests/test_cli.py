"""Config system + command-line trainer (CPU)."""
import json
import os
import subprocess
import sys

import pytest
import yaml

from consensusml_amd.config import TrainConfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_config_yaml_and_overrides(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text(yaml.safe_dump({"agg": {"rule": "krum", "f": 1}, "topology": {"kind": "allgather"},
                                 "model": {"name": "mlp", "extra": {"classes": 3}},
                                 "optim": {"betas": [0.8, 0.9]}}))
    cfg = TrainConfig.from_yaml(str(p)).override(["agg.f=2", "optim.lr=0.5", "fault.ranks=[1,2]"])
    assert cfg.agg.rule == "krum" and cfg.agg.f == 2 and cfg.optim.lr == 0.5
    assert cfg.model.extra == {"classes": 3} and cfg.optim.betas == (0.8, 0.9)
    assert cfg.fault.ranks == [1, 2]
    with pytest.raises(KeyError):
        cfg.override(["agg.nope=1"])
    with pytest.raises(ValueError):
        TrainConfig().override(["agg.rule=bogus"]).validate(4)
    with pytest.raises(ValueError):
        TrainConfig().override(["agg.rule=trimmed_mean", "agg.f=2"]).validate(4)
    d = json.loads(cfg.to_json())
    assert TrainConfig.from_dict({"agg.rule": d["agg"]["rule"]}).agg.rule == "krum"


def test_train_cli_resume(tmp_path):
    out = tmp_path / "res.json"
    args = [sys.executable, "-m", "consensusml_amd.train", "--set", "dtype=fp32",
            "virtual_workers=5", "agg.rule=median", "steps=6", "batch_per_worker=16",
            f"ckpt_dir={tmp_path / 'ck'}", "ckpt_every=3", f"log_path={tmp_path / 'log.jsonl'}",
            "model.extra={classes: 2}", "backend=gloo", "--out", str(out), "--watchdog", "120"]
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run(args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(out.read_text())
    assert res["final_loss"] < 0.7
    assert (tmp_path / "ck" / "latest").exists()
    # resume from step 6 to 9
    args2 = [a if not a.startswith("steps=") else "steps=9" for a in args] + ["--resume"]
    r = subprocess.run(args2, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in (tmp_path / "log.jsonl").read_text().splitlines()]
    assert lines[-1]["step"] == 9


def test_select_cli_synthetic(tmp_path):
    """python -m consensusml_amd.select --synthetic: reference-layout standard table + summary."""
    from consensusml_amd.select.__main__ import main
    out = tmp_path / "sel"
    assert main(["--synthetic", "--genes", "300", "--samples", "48", "--rf-trees", "30",
                 "--lasso-reps", "1", "--device", "cpu", "--out", str(out),
                 "--xgb-configs", '[{"max_depth": 2, "n_estimators": 2}]']) == 0
    assert (out / "standouttable.csv").exists() and (out / "summary.json").exists()


def test_select_cli_counts_with_reference_cohort(tmp_path):
    """--counts path: count columns matched to the reference's own clinical table and split files
    by TARGET USI (synthetic counts, real cohort metadata)."""
    import os
    import numpy as np
    import pandas as pd
    ref = "/root/reference"
    clin = os.path.join(ref, "Clinical_Data", "AML_dataframe.csv")
    if not os.path.exists(clin):
        import pytest
        pytest.skip("reference files not present")
    from consensusml_amd.select.__main__ import main
    from consensusml_amd.select.data import target_aml_cohort
    tr = os.path.join(ref, "JSmith_code", "TARGET_AML_Training_Samples.csv")
    te = os.path.join(ref, "JSmith_code", "TARGET_AML_Testing_Samples.csv")
    co = target_aml_cohort(clin, tr, te)
    usis = list(co.index)
    g = np.random.default_rng(0)
    mat = g.negative_binomial(5, 0.05, size=(250, len(usis))).astype(float)
    low = (co["deg_risk"] == 0).to_numpy()
    mat[:25, low] *= 6.0                     # 25 genes up in Low-risk patients (learnable signal)
    counts = pd.DataFrame(mat.round(), index=[f"ENSG{i:011d}.1" for i in range(250)],
                          columns=[u + "-09A-01R" for u in usis])
    cpath = tmp_path / "counts.csv"
    counts.to_csv(cpath)
    out = tmp_path / "sel"
    assert main(["--counts", str(cpath), "--clinical", clin, "--train-ids", tr, "--test-ids", te,
                 "--rf-trees", "20", "--lasso-reps", "1", "--device", "cpu", "--out", str(out),
                 "--xgb-configs", '[{"max_depth": 2, "n_estimators": 2}]']) == 0
    assert (out / "standouttable.csv").exists()
