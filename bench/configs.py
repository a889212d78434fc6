#!/usr/bin/env python3
"""Runs the BASELINE.json configurations (besides the headline, which is ../bench.py):

  mlp_median      2-layer MLP, coordinate-wise median (CPU/gloo plumbing; any world size)
  resnet_trimmed  ResNet-50 bf16, trimmed-mean aggregation
  resnet_mkrum    ResNet-50 bf16, Multi-Krum
  bert_geomed     BERT-base (MLM, seq 128) bf16, geometric median (Gram-space Weiszfeld)
  llama_gossip    Llama-3-8B bf16, decentralised gossip ring + fused AdamW (seq 2048)

One JSON line per config on rank 0 (throughput = whole-job samples/s and tokens/s, ms/step,
phase breakdown). ``--virtual-workers V`` lets a single GPU aggregate V micro-batch gradients
(robust rules at n = V without more GPUs); default 1 = ranks are the workers.

  python bench/configs.py --config bert_geomed --steps 10 --warmup 3
  torchrun --nproc-per-node 2 --master-addr 127.0.0.1 bench/configs.py --config mlp_median
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CONFIGS = {
    "mlp_median": dict(model="mlp", rule="median", topology="sharded", batch=256, dtype="fp32",
                       optim="sgd", lr=0.1, backend="gloo"),
    "resnet_trimmed": dict(model="resnet50", rule="trimmed_mean", topology="sharded", batch=256,
                           dtype="bf16", optim="sgd", lr=0.1),
    "resnet_mkrum": dict(model="resnet50", rule="multi_krum", topology="sharded", batch=256,
                         dtype="bf16", optim="sgd", lr=0.1),
    "bert_geomed": dict(model="bert_base", rule="geomed", topology="sharded", batch=64,
                        seq_len=128, dtype="bf16", optim="adamw", lr=1e-4),
    # per-GPU batch 4 x 2048 tokens: ~190 GB at world 1 (+16 GB async send buffer at world > 1)
    # of the 288 GB HBM3E; 18.2k tokens/s vs 12.9k at batch 1 (profiles/r01_configs22_llama.jsonl)
    # graph "exp": one peer per step (r + 2^(t mod 3) at N = 8): exact averaging after 3 steps
    # (tests/test_gossip_graphs.py), half the ring's bytes, and ONE 16 GB receive buffer instead
    # of the ring's two (exp_all would need 5 x 16 GB in delayed mode)
    "llama_gossip": dict(model="llama3_8b", rule="mean", topology="gossip", batch=4,
                         seq_len=2048, dtype="bf16", optim="adamw", lr=1e-5, bucket_mb=512,
                         gossip_async=True, gossip_graph="exp"),
}


def default_f(rule: str, n: int) -> int:
    """Byzantine tolerance used when --f is not given: never 0 once the rule can tolerate a
    fault (a robust rule at f = 0 is plain averaging, e.g. Multi-Krum at m = n).
      trimmed_mean   trim (n - 1) // 2 - 1, at least 1 for n >= 3 (n > 2 trim)
      krum / multi_krum / bulyan / others   largest f with n >= 2f + 3, at least 1 for n >= 4
    """
    if rule in ("mean", "median", "geomed"):
        return 0
    if rule == "trimmed_mean":
        return max(1, (n - 1) // 2 - 1) if n >= 3 else 0
    if rule == "bulyan":
        return max(0, (n - 3) // 4)
    return max(1, (n - 3) // 2) if n >= 4 else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=sorted(CONFIGS), required=True)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--virtual-workers", type=int, default=1)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--model", default=None, help="override the model (e.g. llama_tiny)")
    ap.add_argument("--f", type=int, default=-1)
    ap.add_argument("--loopback", action="store_true",
                    help="world 1: run the distributed exchange on a 1-rank process group (RCCL "
                         "send/recv / all-to-all to this rank itself)")
    ap.add_argument("--gossip-graph", default=None, choices=["ring", "exp", "exp_all"])
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--profile-marker", action="store_true",
                    help="launch a spin_kernel between warmup and timed steps (prof_summary --after)")
    a = ap.parse_args()
    c = dict(CONFIGS[a.config])
    if a.model:
        c["model"] = a.model
    from consensusml_amd import TrainConfig, perf
    from consensusml_amd.parallel.dist import init_distributed
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    from consensusml_amd.utils.tuning import configure_miopen
    configure_miopen()
    backend = c.get("backend", "auto")
    if backend == "gloo" and torch.cuda.is_available() and os.environ.get("CML_MLP_GPU") == "1":
        backend = "auto"
    info = init_distributed(backend, loopback=a.loopback)
    torch.backends.cudnn.benchmark = info.device.type == "cuda"
    cfg = TrainConfig()
    cfg.model.name = c["model"]
    cfg.model.seq_len = c.get("seq_len", 128)
    cfg.model.extra = {"classes": 2} if c["model"] == "mlp" else {}
    cfg.batch_per_worker = a.batch or c["batch"]
    cfg.virtual_workers = a.virtual_workers
    n = info.world * a.virtual_workers
    cfg.agg.rule = c["rule"]
    cfg.agg.f = a.f if a.f >= 0 else default_f(c["rule"], n)
    cfg.topology.kind = c["topology"]
    cfg.topology.bucket_mb = c.get("bucket_mb", 64)
    cfg.topology.gossip_async = c.get("gossip_async", False)
    cfg.topology.gossip_graph = a.gossip_graph or c.get("gossip_graph", "ring")
    cfg.dtype = c["dtype"]
    cfg.optim.name = c["optim"]
    cfg.optim.lr = c["lr"]
    cfg.profile = True
    tr = ConsensusTrainer(cfg, info=info)
    sync = torch.cuda.synchronize if info.device.type == "cuda" else (lambda: None)
    for _ in range(a.warmup):
        tr.train_step()
    tr.timer.summary()
    if a.profile_marker and info.device.type == "cuda":
        torch.cuda._sleep(1000)
    sync()
    if info.distributed:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = tr.train_step()
    sync()
    if info.distributed:
        dist.barrier()
    dt = time.perf_counter() - t0
    phases = {k: round(v / a.steps, 3) for k, v in tr.timer.summary().items()}
    if info.distributed:
        t = torch.tensor([dt], dtype=torch.float64, device=info.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
    samples = a.steps * cfg.batch_per_worker * n
    out = {"config": a.config, "model": cfg.model.name, "rule": cfg.agg.rule,
           "topology": cfg.topology.kind, "n_gpus": info.world, "workers": n, "f": cfg.agg.f,
           "per_worker_batch": cfg.batch_per_worker, "dtype": cfg.dtype,
           "optimizer": cfg.optim.name, "params": tr.engine.flat.real_numel,
           "samples_per_s": round(samples / dt, 2),
           "tokens_per_s": round(samples * tr.task.samples_per_item / dt, 1),
           "ms_per_step": round(dt / a.steps * 1e3, 3), "phase_ms_per_step": phases,
           "loss": float(loss), "data": "synthetic", "steps": a.steps, "warmup": a.warmup,
           "batched_workers": bool(n > info.world and tr.task.batched_workers
                                   and perf.policy().batched_workers
                                   and info.device.type == "cuda" and cfg.dtype == "bf16"),
           "perf_policy": perf.policy().to_dict(), "env_switches": perf.env_switches()}
    if info.device.type == "cuda":
        out["max_mem_gb"] = round(torch.cuda.max_memory_allocated() / 2 ** 30, 2)
    out["loopback"] = info.loopback
    if cfg.topology.kind == "gossip":
        e = tr.engine
        out["gossip_graph"] = cfg.topology.gossip_graph
        out["gossip_async"] = cfg.topology.gossip_async
        out["gossip_exchanged"] = bool(e.nb_bufs)
        gb = lambda t: round(t.numel() * t.element_size() / 2 ** 30, 2)   # noqa: E731
        out["memory_plan_gib"] = {
            "params_bf16": gb(e.flat.flat_param), "grads": gb(e.flat.flat_grad),
            "master_fp32": gb(e.master),
            "optimizer_state": round(sum(gb(t) for t in (e.s1, e.s2) if t is not None), 2),
            "neighbour_buffers": round(sum(gb(t) for t in e.nb_bufs), 2),
            "send_buffer": gb(e._send_buf) if e._send_buf is not None else 0.0,
            "n_neighbour_buffers": len(e.nb_bufs)}
    if info.rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "a") as fh:
                fh.write(line + "\n")
    tr.close()
    if info.distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
