#!/usr/bin/env python3
"""Does the fused ResNet-50 step train like the library path?

Three runs from the same random-init weights on a learnable synthetic task (one smooth template
per class + pixel noise, ``models.build_task`` ``synthetic=templates``), same optimizer
(SGD-momentum through the fused HIP update), same data order:

  fused    every own kernel / fusion of the default PerfPolicy (the bench's step)
  library  PerfPolicy.library(): MIOpen / hipBLASLt convolutions + PyTorch BatchNorm
  krum8    the fused step with 8 virtual workers x (batch / 8) and Krum f = 2 (real robust
           aggregation of 8 gradient rows on the one GPU)

Per run: the loss at every step, accuracy after training (train-mode batch statistics and
eval-mode running statistics on fresh batches), and every BN running statistic. The comparison
(fused vs library): loss relative difference at every 10th step, final accuracies, and the
relative difference of the running statistics per BN layer.

  python bench/convergence.py [--steps 100] [--batch 128] [--image-size 224] [--out DIR]
  python bench/convergence.py --steps 30 --batch 2048 --no-krum --noise 2 --noise-floor 0.004
      (the batch-2048 check: the bench's own kernel choices -- M-aware tiles, quad family,
       256 x 256 tiles -- which differ from the small-batch test's)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_cfg(batch: int, image: int, classes: int, lr: float, V: int = 1, rule: str = "mean",
             f: int = 0, seed: int = 7, noise: float = 1.0):
    from consensusml_amd import TrainConfig
    cfg = TrainConfig()
    cfg.model.name = "resnet50"
    cfg.model.num_classes = classes
    cfg.model.image_size = image
    cfg.model.extra = {"synthetic": "templates", "noise": noise}
    cfg.batch_per_worker = batch // V
    cfg.virtual_workers = V
    cfg.agg.rule = rule
    cfg.agg.f = f
    cfg.topology.kind = "sharded"
    cfg.optim.name = "sgd"
    cfg.optim.lr = lr
    cfg.optim.momentum = 0.9
    cfg.optim.weight_decay = 5e-5
    cfg.seed = seed
    cfg.dtype = "bf16"
    return cfg


@torch.no_grad()
def accuracy(tr, batches: int, bs: int, train_mode: bool) -> float:
    """Accuracy on fresh batches of the task (a fixed generator, the same for every run)."""
    tr.engine.wait_params()
    gen = torch.Generator(device=tr.info.device)
    gen.manual_seed(99991)
    m = tr.model
    m.train(train_mode)
    saved = None
    if train_mode:   # train-mode forwards update running statistics: keep them untouched
        saved = [b.clone() for b in m.buffers()]
    hit = tot = 0
    for _ in range(batches):
        x, y = tr.task.make_batch(bs, gen)
        p = m(x).float().argmax(-1)
        hit += int((p == y).sum())
        tot += y.numel()
    if saved is not None:
        for b, s in zip(m.buffers(), saved):
            b.copy_(s)
    m.train(True)
    return hit / tot


def run(name: str, pol, cfg, steps: int, eval_batches: int, eval_bs: int,
        perturb: float = 0.0) -> dict:
    """``perturb`` > 0: multiply every initial master weight by (1 + perturb N(0, 1)) (a fixed
    generator) -- the same model up to rounding-level noise, to measure how far two runs drift
    apart from numerics alone (the noise floor a fused-vs-library difference is judged against)."""
    from consensusml_amd import perf
    from consensusml_amd.parallel.dist import DistInfo
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    dev = torch.device("cuda", 0)
    with perf.use_policy(pol):
        tr = ConsensusTrainer(cfg, info=DistInfo(0, 1, 0, dev, "none"))
        if perturb > 0:
            gen = torch.Generator(device=dev)
            gen.manual_seed(4242)
            m = tr.engine.master
            m.mul_(1 + perturb * torch.randn(m.shape, generator=gen, device=dev))
            tr.engine.sync_params_from_master()
        losses = []
        t0 = time.perf_counter()
        for s in range(steps):
            losses.append(float(tr.train_step()))
            if (s + 1) % 10 == 0 or s < 3:   # early steps too: the first one compiles / finds
                print(f"{name} step {s + 1} loss {losses[-1]:.4f}", flush=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        acc_train = accuracy(tr, eval_batches, eval_bs, True)
        acc_eval = accuracy(tr, eval_batches, eval_bs, False)
        stats = {n: b.float().cpu().clone() for n, b in tr.model.named_buffers()
                 if n.endswith("running_mean") or n.endswith("running_var")}
        sel = tr.engine.sel_counts.cpu().tolist()
        tr.close()
    del tr
    torch.cuda.empty_cache()
    return {"name": name, "losses": losses, "acc_train_mode": acc_train,
            "acc_eval_mode": acc_eval, "stats": stats, "wall_s": dt, "selection_counts": sel}


def compare(a: dict, b: dict, every: int = 10) -> dict:
    """a vs b (b the reference): loss relative differences at every ``every``-th step, accuracy
    differences (points), per-layer relative running-statistics differences."""
    la, lb = a["losses"], b["losses"]
    idx = list(range(every - 1, len(la), every))
    rel = [abs(la[i] - lb[i]) / max(abs(lb[i]), 1e-12) for i in idx]
    # once both runs fit the task the losses are ~1e-3 and their ratio is noise: the tolerance
    # used by the tests is |la - lb| <= 0.1 * max(la, lb) + 0.05 nats
    absd = [abs(la[i] - lb[i]) for i in idx]
    stat_rel = {}
    for k, v in b["stats"].items():
        u = a["stats"][k]
        stat_rel[k] = float((u - v).norm() / v.norm().clamp_min(1e-12))
    return {"steps": [i + 1 for i in idx], "loss_a": [la[i] for i in idx],
            "loss_b": [lb[i] for i in idx], "loss_rel_diff": rel,
            "max_loss_rel_diff": max(rel) if rel else None,
            "mean_loss_abs_diff": sum(absd) / len(absd) if absd else None,
            "acc_train_mode_diff_points": 100 * (a["acc_train_mode"] - b["acc_train_mode"]),
            "acc_eval_mode_diff_points": 100 * (a["acc_eval_mode"] - b["acc_eval_mode"]),
            "bn_stats_max_rel_diff": max(stat_rel.values()),
            "bn_stats_median_rel_diff": sorted(stat_rel.values())[len(stat_rel) // 2],
            "bn_stats_worst_layer": max(stat_rel, key=stat_rel.get)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--classes", type=int, default=10)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--noise", type=float, default=1.0,
                    help="pixel noise over the class templates (higher: a harder task whose loss "
                         "stays informative for longer)")
    ap.add_argument("--eval-batches", type=int, default=8)
    ap.add_argument("--no-krum", action="store_true")
    ap.add_argument("--noise-floor", type=float, default=0.0,
                    help="> 0: also a library run from weights perturbed by this relative amount; "
                         "library vs perturbed-library is the numerics noise floor that the "
                         "fused-vs-library difference is judged against")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from consensusml_amd import perf
    torch.backends.cudnn.benchmark = False     # MIOpen immediate mode: no find for new shapes
    fused_pol = perf.policy()
    runs = {}
    runs["fused"] = run("fused", fused_pol,
                        make_cfg(a.batch, a.image_size, a.classes, a.lr, noise=a.noise),
                        a.steps, a.eval_batches, a.batch)
    runs["library"] = run("library", perf.PerfPolicy.library(),
                          make_cfg(a.batch, a.image_size, a.classes, a.lr, noise=a.noise), a.steps,
                          a.eval_batches, a.batch)
    if a.noise_floor > 0:
        runs["library_perturbed"] = run("library_perturbed", perf.PerfPolicy.library(),
                                        make_cfg(a.batch, a.image_size, a.classes, a.lr,
                                                 noise=a.noise), a.steps, a.eval_batches,
                                        a.batch, perturb=a.noise_floor)
    if not a.no_krum:
        runs["krum8"] = run("krum8", fused_pol,
                            make_cfg(a.batch, a.image_size, a.classes, a.lr, V=8, rule="krum",
                                     f=2, noise=a.noise), a.steps, a.eval_batches, a.batch)
    cmp = compare(runs["fused"], runs["library"])
    floor = compare(runs["library_perturbed"], runs["library"]) if a.noise_floor > 0 else None
    summary = {"config": vars(a), "fused_vs_library": cmp, "noise_floor": floor,
               "runs": {k: {kk: vv for kk, vv in r.items() if kk != "stats"}
                        for k, r in runs.items()}}
    line = json.dumps(summary)
    print(json.dumps({"fused_vs_library": {k: v for k, v in cmp.items()
                                            if not isinstance(v, list)},
                      "noise_floor": ({k: v for k, v in floor.items() if not isinstance(v, list)}
                                      if floor else None),
                      "final_loss": {k: r["losses"][-1] for k, r in runs.items()},
                      "acc_eval_mode": {k: r["acc_eval_mode"] for k, r in runs.items()},
                      "acc_train_mode": {k: r["acc_train_mode"] for k, r in runs.items()},
                      "wall_s": {k: round(r["wall_s"], 1) for k, r in runs.items()}}),
          flush=True)
    if a.out:
        os.makedirs(a.out, exist_ok=True)
        with open(os.path.join(a.out, "convergence.json"), "w") as fh:
            fh.write(line + "\n")
        with open(os.path.join(a.out, "curves.csv"), "w") as fh:
            names = list(runs)
            fh.write("step," + ",".join(f"loss_{n}" for n in names) + "\n")
            for s in range(a.steps):
                fh.write(f"{s + 1}," + ",".join(f"{runs[n]['losses'][s]:.6f}" for n in names)
                         + "\n")


if __name__ == "__main__":
    main()
