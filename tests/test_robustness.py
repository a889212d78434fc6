"""Qualitative outcomes of the robustness benchmark (bench/robustness.py) on CPU: n = 8 virtual
workers, 2 Byzantine from step 0, MLP on a learnable teacher task. The full rule x attack table
(MLP and resnet_tiny, on the GPU kernels) is profiles/r02_robustness.md."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "bench"))
from robustness import alie_z, markdown, run_one  # noqa: E402

STEPS = 150
CPU = torch.device("cpu")


def _run(rule, attack):
    return run_one("mlp", rule, attack, n=8, f=2, steps=STEPS, device=CPU)


def test_alie_z_matches_paper():
    # Baruch et al. 2019: n = 50, f = 12 -> s = 14, z = Phi^-1(36/50) ~ 0.58
    assert abs(alie_z(50, 12) - 0.5828) < 1e-3
    assert abs(alie_z(8, 2) - 0.3186) < 1e-3


def test_clean_baseline_learns():
    r = _run("mean", "none")
    assert r["eval_accuracy"] > 0.85 and r["final_train_loss"] < 0.5 * r["initial_loss"]


@pytest.mark.parametrize("attack", ["sign_flip", "scaled"])
def test_mean_breaks(attack):
    r = _run("mean", attack)
    assert r["diverged"] or r["eval_accuracy"] < 0.5, r


@pytest.mark.parametrize("rule", ["median", "trimmed_mean", "geomed", "multi_krum",
                                  "centered_clip"])
@pytest.mark.parametrize("attack", ["sign_flip", "scaled"])
def test_robust_rules_bounded(rule, attack):
    r = _run(rule, attack)
    assert not r["diverged"]
    assert r["eval_accuracy"] > 0.8, r
    assert r["final_train_loss"] < 0.5 * r["initial_loss"], r
    if rule == "multi_krum":
        assert r["byzantine_selected_frac"] == 0.0


def test_krum_ipm_known_failure():
    """Documented failure mode: the two IPM colluders send the same small vector (-0.1 mu), so
    they are each other's nearest neighbour and Krum picks one of them almost every step; the
    model is then driven uphill. Multi-Krum (averaging n - f) and the coordinate-wise rules
    survive the same attack."""
    k = _run("krum", "ipm")
    assert k["byzantine_selected_frac"] > 0.8
    assert k["eval_accuracy"] < 0.5
    m = _run("multi_krum", "ipm")
    assert m["eval_accuracy"] > 0.8


def test_markdown_table():
    rows = [_run("median", "none"), _run("median", "sign_flip")]
    md = markdown(rows)
    assert "| median |" in md and "sign_flip (g*-10)" in md


@pytest.mark.gpu
def test_gpu_robustness_cells(cuda):
    """The same qualitative outcomes on the HIP aggregation / fault / update kernels (bf16)."""
    def run(rule, attack):
        return run_one("mlp", rule, attack, n=8, f=2, steps=STEPS, device=cuda)
    assert run("mean", "none")["eval_accuracy"] > 0.8
    r = run("mean", "sign_flip")
    assert r["diverged"] or r["eval_accuracy"] < 0.5
    for rule in ("median", "trimmed_mean", "geomed", "bulyan"):
        r = run(rule, "sign_flip")
        assert not r["diverged"] and r["eval_accuracy"] > 0.8, r
    assert run("krum", "ipm")["byzantine_selected_frac"] > 0.8
