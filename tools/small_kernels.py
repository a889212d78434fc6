#!/usr/bin/env python3
"""Where do the small launches of a training step come from?

Profiles one bench step (torch.profiler, CPU + CUDA activities, Python stacks) and attributes every
device kernel to the ATen op that launched it and to the innermost ``consensusml_amd`` frame of
that op's Python stack. Prints launches per step and device time per call site, largest count
first, so the per-layer glue (dtype conversions, concatenations, weight transposes, fills) can be
found and fused.

  python tools/small_kernels.py --batch 256 [--model resnet50] [--top 40] > gpurun_out/small.txt
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--virtual-workers", type=int, default=1)
    ap.add_argument("--rule", default="krum")
    ap.add_argument("--seq-len", type=int, default=128)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    from consensusml_amd import TrainConfig
    from consensusml_amd.parallel.dist import DistInfo
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    from consensusml_amd.utils.tuning import configure_miopen
    configure_miopen()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    cfg = TrainConfig()
    cfg.model.name = a.model
    cfg.model.seq_len = a.seq_len
    cfg.batch_per_worker = a.batch
    cfg.virtual_workers = a.virtual_workers
    cfg.agg.rule = a.rule
    cfg.agg.f = 1 if a.rule in ("krum", "multi_krum") and a.virtual_workers >= 4 else 0
    cfg.topology.kind = "sharded"
    cfg.optim.name = "sgd" if a.model.startswith("resnet") else "adamw"
    tr = ConsensusTrainer(cfg, info=DistInfo(0, 1, 0, dev, "none"))
    for _ in range(3):
        tr.train_step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        tr.train_step()
        torch.cuda.synchronize()
    events = prof.events()
    # every CPU op's own kernels (Kineto correlates each launch with the innermost op), keyed by
    # the op and its innermost consensusml_amd frame
    by = collections.defaultdict(lambda: [0, 0.0])
    kernels = 0
    total_us = 0.0
    for e in events:
        if e.device_type.name != "CPU" or not getattr(e, "kernels", None):
            continue
        # innermost package frame on this op's or an enclosing op's stack; backward ops run on the
        # autograd thread (no Python stack): name the enclosing autograd Function / op chain
        where, p, chain = None, e, []
        while p is not None and where is None:
            fr = [s for s in (p.stack or []) if "consensusml_amd" in s]
            if fr:
                where = fr[0].split("consensusml_amd/")[-1]
            else:
                chain.append(p.name)
                p = getattr(p, "cpu_parent", None)
        if where is None:
            fn = [n for n in chain if "Backward" in n or n.startswith("_")]
            where = fn[0] if fn else " < ".join(chain[:3])
        for k in e.kernels:
            kernels += 1
            total_us += k.duration
            rec = by[(e.name, where, k.name[:60])]
            rec[0] += 1
            rec[1] += k.duration
    print(f"kernels per step: {kernels}, device time {total_us / 1e3:.2f} ms")
    rows = sorted(by.items(), key=lambda kv: -kv[1][0])
    print(f"{'count':>6} {'ms':>8}  op | call site | kernel")
    for (op, where, kname), (n, us) in rows[:a.top]:
        print(f"{n:6d} {us / 1e3:8.3f}  {op} | {where} | {kname}")


if __name__ == "__main__":
    main()
