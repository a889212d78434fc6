#!/usr/bin/env python3
"""Attribute the small fill / MIOpen SetTensor kernels of the ResNet-50 bench step to the ATen ops
that launch them (torch.profiler with Python stacks), to see which of them our own code causes.

  python tools/torch_prof_fills.py --batch 512 > gpurun_out/fills.txt
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--keys", default="fill,zero,SubTensor,Memset,memset",
                    help="comma-separated substrings of the op names to attribute")
    a = ap.parse_args()
    from consensusml_amd import TrainConfig
    from consensusml_amd.parallel.dist import DistInfo
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    from consensusml_amd.utils.tuning import configure_miopen
    configure_miopen()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    cfg = TrainConfig()
    cfg.model.name = "resnet50"
    cfg.batch_per_worker = a.batch
    cfg.agg.rule = "krum"
    cfg.topology.kind = "sharded"
    cfg.optim.name = "sgd"
    tr = ConsensusTrainer(cfg, info=DistInfo(0, 1, 0, dev, "none"))
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    batch = tr.task.make_batch(a.batch, gen)

    def step():
        tr.engine.zero_grad()
        tr.task.loss_fn(tr.model, batch).backward()
        tr.engine.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    keys = tuple(a.keys.split(","))
    print(prof.key_averages(group_by_stack_n=6).table(sort_by="self_device_time_total",
                                                      row_limit=60, max_name_column_width=60))
    print("=== ops containing", keys, "===")
    for e in prof.key_averages(group_by_input_shape=True):
        if any(k in e.key for k in keys) and e.self_device_time_total > 0:
            print(e.key, e.count, round(e.self_device_time_total / 1e3, 3), "ms", e.input_shapes)
    for e in prof.key_averages(group_by_stack_n=8):
        if any(k in e.key for k in keys) and e.self_device_time_total > 0:
            print(e.key, e.count, round(e.self_device_time_total / 1e3, 3), "ms")
            for fr in e.stack[:8]:
                print("     ", fr)


if __name__ == "__main__":
    main()
