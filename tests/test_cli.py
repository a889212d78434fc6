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
