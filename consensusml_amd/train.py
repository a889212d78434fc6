"""Command-line trainer: ``python -m consensusml_amd.train --config cfg.yaml --set agg.rule=krum``.

Launch multi-GPU with ``torchrun --nproc-per-node N --master-addr 127.0.0.1 -m
consensusml_amd.train ...`` (one process per GPU, RCCL). Writes JSONL step logs
(``log_path``), checkpoints (``ckpt_dir`` / ``ckpt_every``, resumable with ``--resume``) and
a final result JSON on rank 0. A native watchdog (``--watchdog SECONDS``) reports, and with
``--watchdog-abort`` kills, a rank that stops making progress (hung collective).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

from .config import add_cli, from_cli


def main(argv=None) -> int:
    ap = add_cli(argparse.ArgumentParser(description=__doc__))
    ap.add_argument("--resume", action="store_true")
    ap.add_argument("--out", default=None, help="result JSON (rank 0)")
    ap.add_argument("--watchdog", type=float, default=0.0)
    ap.add_argument("--watchdog-abort", action="store_true")
    ap.add_argument("--eval-batches", type=int, default=2)
    ap.add_argument("--conv-find", action="store_true",
                    help="MIOpen find mode for convolutions (shipped find-db, no naive solvers)")
    a = ap.parse_args(argv)
    cfg = from_cli(a)
    if a.conv_find:
        import torch
        from .utils.tuning import configure_miopen
        configure_miopen()
        torch.backends.cudnn.benchmark = True
    from .parallel.dist import init_distributed, shutdown
    from .trainer.trainer import ConsensusTrainer
    info = init_distributed(cfg.backend)
    tr = ConsensusTrainer(cfg, info=info)
    wd = None
    if a.watchdog > 0:
        from .runtime import Watchdog
        rep = (cfg.log_path or "watchdog") + f".rank{info.rank}.watchdog.jsonl"
        wd = Watchdog(a.watchdog, rep, a.watchdog_abort)
    if a.resume and cfg.ckpt_dir:
        from .trainer.checkpoint import latest_checkpoint
        if latest_checkpoint(cfg.ckpt_dir):
            tr.load(cfg.ckpt_dir)
    res = {}
    start = tr.engine.step_count
    stats_ok = tr.engine.topo in ("sharded", "allgather")
    for s in range(start, cfg.steps):
        ckpt_now = bool(cfg.ckpt_every and cfg.ckpt_dir and (s + 1) % cfg.ckpt_every == 0)
        if stats_ok and ckpt_now:
            tr.engine.record_stats = True     # the checkpoint's consensus_table.csv
        loss = tr.train_step()
        if wd is not None:
            wd.beat(s)
        if (s + 1) % 10 == 0 or s + 1 == cfg.steps:
            tr.logger.log(step=s + 1, loss=float(loss), selection=tr.engine.sel_counts.tolist())
        if ckpt_now:
            tr.save()
    res["final_loss"] = float(loss) if cfg.steps > start else None
    res["eval"] = tr.evaluate(a.eval_batches)
    res["selection_counts"] = tr.engine.sel_counts.tolist()
    res["config"] = json.loads(cfg.to_json())
    if wd is not None:
        wd.stop()
    if info.rank == 0:
        line = json.dumps(res, default=str)
        print(line)
        if a.out:
            with open(a.out, "w") as fh:
                fh.write(line + "\n")
    tr.close()
    shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
