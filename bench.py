#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 bf16 data-parallel training with Krum consensus aggregation.

BASELINE.json metric: "samples/sec ResNet-50 + Krum at 1/2/4/8 MI355X; agg overhead vs
all-reduce". One process per GPU (``python -m torch.distributed.run --nproc-per-node N
--master-addr 127.0.0.1 bench.py --gpus N``), RCCL over xGMI, weak scaling (fixed per-GPU
batch). Each rank is one Krum worker; the default topology is the sharded ("robust ZeRO")
exchange: bucketed all-to-all of bf16 gradients overlapped with backward -> per-shard MFMA Gram
-> all-reduce of the n x n Gram -> Krum weights -> fused weighted-sum + SGD-momentum update of
the fp32 master shard -> all-gather of bf16 parameters. After the timed Krum run, the same
model/batch runs with the plain mean all-reduce baseline (DDP-equivalent, same fused optimizer)
and ``agg_overhead_vs_allreduce`` = (t_krum - t_allreduce) / t_allreduce is reported.

Data: synthetic ImageNet-shaped batches (random bf16 images, random labels) generated on
device; random-init weights. Every timed step runs the full forward, backward, exchange,
aggregation and optimizer update. Per-GPU batch 2048 by default: 288 GB of HBM holds it many times
over (peak ~81 GiB), and throughput still rises with batch (512 ~11.5k, 1024 ~12.0k, 1536
~12.1-12.4k, 2048 ~12.3k samples/s: larger conv / GEMM problems, fewer fixed per-step costs).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

METRIC = "samples/sec ResNet-50 + Krum at 1/2/4/8 MI355X; agg overhead vs all-reduce"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=2048,
                    help="per-GPU batch (samples/s on MI355X: 512 ~11.5k, 1024 ~12.0k, 1536 "
                         "~12.1-12.4k, 2048 ~12.3k, profiles/r01_bench55/66/69_b*.json; peak memory "
                         "~81 GiB at 2048 of 288; the shipped MIOpen find-db covers all four)")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--rule", default="krum")
    ap.add_argument("--f", type=int, default=-1, help="Byzantine tolerance (-1: (n-3)//2)")
    ap.add_argument("--topology", default="sharded")
    ap.add_argument("--bucket-mb", type=float, default=25.0)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--no-baseline", action="store_true")
    ap.add_argument("--baseline-steps", type=int, default=-1)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 (nccl = RCCL; gloo only to rehearse "
                         "several ranks sharing one GPU)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--conv1x1", choices=["auto", "gemm", "miopen"], default="auto",
                    help="1x1 stride-1 conv forward / data gradient as hipBLASLt GEMMs: per-shape "
                         "measured choice (auto), always, or never (MIOpen)")
    ap.add_argument("--profile-marker", action="store_true",
                    help="launch a spin_kernel between warmup and timed steps (prof_summary --after)")
    ap.add_argument("--no-miopen-find", action="store_true",
                    help="disable MIOpen find mode (torch.backends.cudnn.benchmark) for convs")
    return ap.parse_args()


def run(args, rule: str, topology: str, steps: int, warmup: int, info):
    from consensusml_amd.parallel.dist import barrier
    from consensusml_amd import TrainConfig
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    n = info.world
    cfg = TrainConfig()
    cfg.model.name = args.model
    cfg.model.image_size = args.image_size
    cfg.batch_per_worker = args.batch
    cfg.dtype = "bf16"
    cfg.agg.rule = rule
    cfg.agg.f = args.f if args.f >= 0 else max(0, (n - 3) // 2)
    cfg.topology.kind = topology
    cfg.topology.bucket_mb = args.bucket_mb
    cfg.topology.overlap = not args.no_overlap
    cfg.optim.name = "sgd"
    cfg.optim.lr = 0.1
    cfg.optim.momentum = 0.9
    cfg.optim.weight_decay = 5e-5
    tr = ConsensusTrainer(cfg, info=info)
    dev = info.device
    # pre-generate a few synthetic batches (data generation is not part of the step)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + info.rank)
    batches = [tr.task.make_batch(args.batch, gen) for _ in range(2)]
    model, eng = tr.model, tr.engine

    def step(i):
        eng.zero_grad()
        loss = tr.task.loss_fn(model, batches[i % len(batches)])
        loss.backward()
        eng.step()
        return loss

    tw = time.perf_counter()
    for i in range(max(warmup, 1 if torch.backends.cudnn.benchmark else 0)):
        step(i)
        if info.rank == 0:   # progress: a cold MIOpen find for new conv shapes can take minutes
            torch.cuda.synchronize()
            print(f"[bench] {rule}/{topology}: warmup step {i} done at {time.perf_counter() - tw:.1f}s",
                  file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if info.rank == 0:
        print(f"[bench] {rule}/{topology}: warmup {time.perf_counter() - tw:.1f}s", file=sys.stderr,
              flush=True)
    if args.profile_marker:
        torch.cuda._sleep(1000)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        loss = step(i)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if info.distributed:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    finite = bool(torch.isfinite(loss).item())
    res = {"dt": dt, "f": cfg.agg.f, "loss": float(loss.item()), "finite": finite,
           "params": eng.flat.real_numel, "buckets": len(eng.flat.buckets)}
    tr.close()
    del tr, eng, model, batches
    torch.cuda.empty_cache()
    return res


def main():
    args = parse()
    from consensusml_amd.models import resnet as _resnet
    _resnet.CONV1X1_GEMM = args.conv1x1
    if not args.no_miopen_find:
        from consensusml_amd.utils.tuning import configure_miopen
        configure_miopen()
    from consensusml_amd.parallel.dist import init_distributed
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={world_env}", file=sys.stderr)
    info = init_distributed(args.dist_backend if world_env > 1 else "auto",
                            device="cuda:0" if args.dist_backend == "gloo" else None)
    # MIOpen find mode: conv solvers are benchmarked on first use of each shape (untimed: the
    # warmup steps, plus one tuning step when --warmup 0) and cached for the run.
    torch.backends.cudnn.benchmark = not args.no_miopen_find
    n = info.world
    main_res = run(args, args.rule, args.topology, args.steps, args.warmup, info)
    ms = main_res["dt"] / args.steps * 1e3
    value = n * args.batch * args.steps / main_res["dt"]
    overhead = None
    base_ms = None
    if not args.no_baseline:
        bsteps = args.baseline_steps if args.baseline_steps > 0 else args.steps
        base = run(args, "mean", "allreduce", bsteps, args.warmup, info)
        base_ms = base["dt"] / bsteps * 1e3
        overhead = (ms - base_ms) / base_ms
    if info.rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "samples/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random bf16 224x224 images + labels on device; random-init weights)",
            "config": {"model": "resnet50", "global_batch": n * args.batch, "seq_len": None,
                       "image_size": args.image_size, "per_gpu_batch": args.batch,
                       "parallelism": f"dp{n}", "rule": args.rule, "f": main_res["f"],
                       "topology": args.topology, "optimizer": "sgd-momentum (fused HIP)",
                       "conv1x1": args.conv1x1,
                       "params": main_res["params"], "buckets": main_res["buckets"]},
            "allreduce_ms_per_step": None if base_ms is None else round(base_ms, 3),
            "agg_overhead_vs_allreduce": None if overhead is None else round(overhead, 4),
            "loss_finite": main_res["finite"],
            "peak_mem_gib": (round(torch.cuda.max_memory_allocated() / 2**30, 1)
                             if torch.cuda.is_available() else None),
        }
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as fh:
                fh.write(line + "\n")
    if info.distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
