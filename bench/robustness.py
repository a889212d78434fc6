#!/usr/bin/env python3
"""Robustness benchmark: aggregation rule x Byzantine attack -> final loss and accuracy.

The product claim of the reference framework is that a consensus rule keeps training on course
when some workers lie. This runs it: n = 8 workers simulated as virtual
workers on one device (each has its own data stream and gradient row, exactly as a rank would),
f = 2 of them Byzantine from step 0, on two learnable synthetic tasks:

  mlp          32 -> 64 -> 10 MLP, labels = argmax of a fixed random linear teacher
  resnet_tiny  ResNet (width 8, one block per stage) on 32x32 images: one smooth template per
               class plus pixel noise 6x its scale (models.build_task extra synthetic=templates)

Rules:   mean, median, trimmed_mean (trim f), krum (f), multi_krum (m = n - f), geomed,
         bulyan (f = (n - 3) // 4 = 1: the rule needs n >= 4f + 3, so at n = 8 it is configured
         for one fault while two attack -- reported as such), centered_clip (tau, 3 iterations)
Attacks: none, sign_flip (g <- -10 g), gaussian (g <- N(0, sigma^2)), scaled (g <- 100 g),
         alie (mu - z sigma of the honest workers, z from Baruch et al. 2019: z_max for n, f),
         ipm (-eps * mu, eps = 0.1, Xie et al. 2020)

Every cell reports the mean training loss of the last 10 steps (the loss of the honest workers'
batches at the current model), held-out loss / accuracy on 8 fresh batches, whether the run
diverged (non-finite), and for Krum / Multi-Krum how often a Byzantine worker was selected.

  python bench/robustness.py --task mlp --steps 200 --jsonl out.jsonl --md out.md
  python bench/robustness.py --task resnet_tiny --rules krum,median --attacks alie
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from statistics import NormalDist
from typing import Dict, List, Optional

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

RULES = ("mean", "median", "trimmed_mean", "krum", "multi_krum", "geomed", "bulyan",
         "centered_clip")
ATTACKS = ("none", "sign_flip", "gaussian", "scaled", "alie", "ipm")

TASKS = {
    "mlp": dict(model="mlp", in_features=32, hidden=64, classes=10, batch=32, lr=0.05,
                steps=200),
    # pixel noise 6x the template scale: at noise 1 every rule reaches ~100 % and the attacks
    # only show up in the loss (profiles/r02_robustness/table_noise1.md)
    "resnet_tiny": dict(model="resnet_tiny", classes=10, image_size=32, batch=32, lr=0.05,
                        steps=150, noise=6.0),
}


def alie_z(n: int, f: int) -> float:
    """z_max of "A Little Is Enough": s = floor(n/2 + 1) - f supporters needed, z = Phi^-1((n-s)/n)."""
    s = n // 2 + 1 - f
    return NormalDist().inv_cdf((n - s) / n)


def rule_f(rule: str, n: int, f: int) -> int:
    if rule == "bulyan":
        return min(f, max(0, (n - 3) // 4))
    return f


def make_config(task: str, rule: str, attack: str, n: int = 8, f: int = 2,
                steps: Optional[int] = None, dtype: str = "bf16", tau: float = 1.0,
                seed: int = 2019):
    from consensusml_amd import TrainConfig
    t = TASKS[task]
    cfg = TrainConfig()
    cfg.seed = seed
    cfg.dtype = dtype
    cfg.model.name = t["model"]
    if t["model"] == "mlp":
        cfg.model.in_features = t["in_features"]
        cfg.model.hidden = t["hidden"]
        cfg.model.extra = {"classes": t["classes"]}
    else:
        cfg.model.num_classes = t["classes"]
        cfg.model.image_size = t["image_size"]
        cfg.model.extra = {"synthetic": "templates", "noise": t["noise"]}
    cfg.batch_per_worker = t["batch"]
    cfg.virtual_workers = n
    cfg.steps = steps or t["steps"]
    cfg.agg.rule = rule
    cfg.agg.f = rule_f(rule, n, f)
    cfg.agg.tau = tau
    cfg.topology.kind = "sharded"
    cfg.optim.name = "sgd"
    cfg.optim.lr = t["lr"]
    cfg.optim.momentum = 0.9
    cfg.fault.kind = attack
    cfg.fault.ranks = list(range(f)) if attack != "none" else []
    if attack == "sign_flip":
        cfg.fault.scale = 10.0
    elif attack == "scaled":
        cfg.fault.scale = 100.0
    elif attack == "gaussian":
        cfg.fault.sigma = 1.0
    elif attack == "alie":
        cfg.fault.z = alie_z(n, f)
    elif attack == "ipm":
        cfg.fault.scale = 0.1
    return cfg


def fault_desc(cfg) -> str:
    k = cfg.fault.kind
    return {"none": "-", "sign_flip": f"g*-{cfg.fault.scale:g}", "scaled": f"g*{cfg.fault.scale:g}",
            "gaussian": f"N(0,{cfg.fault.sigma:g}^2)", "alie": f"z={cfg.fault.z:.3f}",
            "ipm": f"eps={cfg.fault.scale:g}"}[k]


def run_one(task: str, rule: str, attack: str, n: int = 8, f: int = 2,
            steps: Optional[int] = None, device: Optional[torch.device] = None,
            dtype: Optional[str] = None, tau: float = 1.0, seed: int = 2019) -> Dict[str, object]:
    from consensusml_amd.parallel.dist import DistInfo
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    if device is None:
        device = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    if dtype is None:
        dtype = "bf16" if device.type == "cuda" else "fp32"
    cfg = make_config(task, rule, attack, n, f, steps, dtype, tau, seed)
    tr = ConsensusTrainer(cfg, info=DistInfo(0, 1, 0, device, "none"))
    t0 = time.perf_counter()
    res = tr.fit(cfg.steps, log_every=0)
    wall = time.perf_counter() - t0
    ev = tr.evaluate(batches=8, batch_size=256)
    hist = res["history"]
    tail = hist[-10:]
    final = sum(tail) / len(tail)
    finite = all(math.isfinite(h) for h in tail) and math.isfinite(ev["loss"])
    sel = res["selection_counts"]
    byz = cfg.fault.ranks
    out = {"task": task, "rule": rule, "attack": attack, "attack_params": fault_desc(cfg),
           "n": n, "f": f, "f_attackers": len(byz), "f_rule": cfg.agg.f, "steps": cfg.steps,
           "dtype": dtype, "device": device.type,
           "initial_loss": hist[0], "final_train_loss": final, "eval_loss": ev["loss"],
           "eval_accuracy": ev["accuracy"], "diverged": not finite, "wall_s": round(wall, 2)}
    if rule in ("krum", "multi_krum"):
        tot = sum(sel)
        out["byzantine_selected_frac"] = (sum(sel[b] for b in byz) / tot) if tot else 0.0
    if rule == "centered_clip":
        out["tau"] = tau
    tr.close()
    return out


def markdown(rows: List[Dict[str, object]]) -> str:
    """accuracy (and final train loss) table per task: rules down, attacks across."""
    lines = []
    for task in sorted({r["task"] for r in rows}):
        rs = [r for r in rows if r["task"] == task]
        attacks = [a for a in ATTACKS if any(r["attack"] == a for r in rs)]
        rules = [u for u in RULES if any(r["rule"] == u for r in rs)]
        params = {r["attack"]: r["attack_params"] for r in rs}
        r0 = rs[0]
        lines.append(f"### {task}: n = {r0['n']} workers, {r0.get('f', 2)} Byzantine, "
                     f"{r0['steps']} steps, {r0['dtype']} on {r0['device']}")
        lines.append("")
        lines.append("Held-out accuracy / final training loss (mean of the last 10 steps); "
                     "`DIV` = diverged (non-finite).")
        lines.append("")
        lines.append("| rule | " + " | ".join(f"{a} ({params[a]})" for a in attacks) + " |")
        lines.append("|---|" + "---|" * len(attacks))
        for u in rules:
            cells = []
            for a in attacks:
                m = [r for r in rs if r["rule"] == u and r["attack"] == a]
                if not m:
                    cells.append("")
                    continue
                r = m[0]
                if r["diverged"]:
                    cells.append("DIV")
                    continue
                c = f"{r['eval_accuracy']:.3f} / {r['final_train_loss']:.3f}"
                if "byzantine_selected_frac" in r and a != "none":
                    c += f" (byz sel {r['byzantine_selected_frac']:.2f})"
                cells.append(c)
            label = u if u != "bulyan" else "bulyan (f=1)"
            lines.append(f"| {label} | " + " | ".join(cells) + " |")
        lines.append("")
    return "\n".join(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", choices=sorted(TASKS), default="mlp")
    ap.add_argument("--rules", default=",".join(RULES))
    ap.add_argument("--attacks", default=",".join(ATTACKS))
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--f", type=int, default=2)
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--tau", type=float, default=1.0)
    ap.add_argument("--device", default=None)
    ap.add_argument("--dtype", default=None)
    ap.add_argument("--jsonl", default=None)
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    dev = torch.device(a.device) if a.device else None
    rows = []
    for rule in a.rules.split(","):
        for attack in a.attacks.split(","):
            r = run_one(a.task, rule, attack, a.n, a.f, a.steps or None, dev, a.dtype, a.tau)
            rows.append(r)
            line = json.dumps(r)
            print(line, flush=True)
            if a.jsonl:
                with open(a.jsonl, "a") as fh:
                    fh.write(line + "\n")
    if a.md:
        with open(a.md, "a") as fh:
            fh.write(markdown(rows) + "\n")


if __name__ == "__main__":
    main()
