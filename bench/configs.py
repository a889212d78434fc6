#!/usr/bin/env python3
"""Runs the BASELINE.json configurations (besides the headline, which is ../bench.py) under the
headline harness's contract:

  mlp_median      2-layer MLP, coordinate-wise median (CPU/gloo plumbing; any world size)
  resnet_trimmed  ResNet-50 bf16, trimmed-mean aggregation
  resnet_mkrum    ResNet-50 bf16, Multi-Krum
  bert_geomed     BERT-base (MLM, seq 128) bf16, geometric median (Gram-space Weiszfeld)
  llama_gossip    Llama-3-8B bf16, decentralised gossip + fused AdamW (seq 2048)

Contract (as bench.py): ``--gpus N`` one process per GPU -- self-launched when no launcher set
WORLD_SIZE, exit 2 on a world-size mismatch; W untimed warmup steps, then K timed steps
bracketed by barrier + synchronize on both sides, the MAX over ranks; after the config's own run
the same model / batch / optimizer runs with the plain mean all-reduce (DDP-equivalent) baseline
and ``agg_overhead_vs_allreduce`` = (t_rule - t_allreduce) / t_allreduce is reported;
``replicas_identical`` is a cross-rank bitwise parameter check (null for gossip, whose replicas
only agree after averaging). Gradient buckets default to 8 MB for the all-to-all configs (the
last bucket's exchange cannot hide behind backward). One JSON line per config on rank 0
(whole-job samples/s and tokens/s, ms/step, phase breakdown). ``--virtual-workers V`` lets a
single GPU aggregate V micro-batch gradients (robust rules at n = V without more GPUs).

  python bench/configs.py --config bert_geomed --steps 10 --warmup 3
  python bench/configs.py --config resnet_mkrum --gpus 8
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {
    "mlp_median": dict(model="mlp", rule="median", topology="sharded", batch=256, dtype="fp32",
                       optim="sgd", lr=0.1, backend="gloo", bucket_mb=8),
    "resnet_trimmed": dict(model="resnet50", rule="trimmed_mean", topology="sharded", batch=256,
                           dtype="bf16", optim="sgd", lr=0.1, bucket_mb=8),
    "resnet_mkrum": dict(model="resnet50", rule="multi_krum", topology="sharded", batch=256,
                         dtype="bf16", optim="sgd", lr=0.1, bucket_mb=8),
    "bert_geomed": dict(model="bert_base", rule="geomed", topology="sharded", batch=64,
                        seq_len=128, dtype="bf16", optim="adamw", lr=1e-4, bucket_mb=8),
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


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=sorted(CONFIGS), required=True)
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without WORLD_SIZE, N > 1 self-launches N ranks")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--virtual-workers", type=int, default=1)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--model", default=None, help="override the model (e.g. llama_tiny)")
    ap.add_argument("--seq-len", type=int, default=0, help="override the sequence length")
    ap.add_argument("--f", type=int, default=-1)
    ap.add_argument("--no-direct-grads", action="store_true",
                    help="copy-on-ready gradient capture even where ops can write the flat row")
    ap.add_argument("--bucket-mb", type=float, default=0.0, help="0: the config's default")
    ap.add_argument("--no-baseline", action="store_true",
                    help="skip the mean all-reduce baseline run")
    ap.add_argument("--loopback", action="store_true",
                    help="world 1: run the distributed exchange on a 1-rank process group (RCCL "
                         "send/recv / all-to-all to this rank itself)")
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="auto: the config's backend (gloo for mlp_median), else nccl on GPU")
    ap.add_argument("--gossip-graph", default=None, choices=["ring", "exp", "exp_all"])
    ap.add_argument("--timeout", type=float, default=900.0,
                    help="seconds any collective may block before the run fails")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--profile-marker", action="store_true",
                    help="launch a spin_kernel between warmup and timed steps (prof_summary --after)")
    return ap.parse_args(argv)


def run_config(c: dict, a, info, rule: str, topology: str) -> dict:
    """Build a trainer for config c with (rule, topology), W warmup + K timed steps."""
    from consensusml_amd import TrainConfig, perf
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    from consensusml_amd.utils.launch import replicas_identical
    cfg = TrainConfig()
    cfg.model.name = c["model"]
    cfg.model.seq_len = a.seq_len or c.get("seq_len", 128)
    cfg.model.extra = {"classes": 2} if c["model"] == "mlp" else {}
    cfg.batch_per_worker = a.batch or c["batch"]
    cfg.virtual_workers = a.virtual_workers
    n = info.world * a.virtual_workers
    cfg.agg.rule = rule
    cfg.agg.f = 0 if rule == "mean" else (a.f if a.f >= 0 else default_f(rule, n))
    cfg.topology.kind = topology
    cfg.topology.direct_grads = not a.no_direct_grads
    cfg.topology.bucket_mb = a.bucket_mb or c.get("bucket_mb", 8)
    cfg.topology.gossip_async = c.get("gossip_async", False)
    cfg.topology.gossip_graph = a.gossip_graph or c.get("gossip_graph", "ring")
    cfg.dtype = c["dtype"]
    cfg.optim.name = c["optim"]
    cfg.optim.lr = c["lr"]
    cfg.profile = True
    tr = ConsensusTrainer(cfg, info=info)
    cuda = info.device.type == "cuda"
    sync = torch.cuda.synchronize if cuda else (lambda: None)
    for i in range(a.warmup):
        tr.train_step()
        if info.rank == 0:
            sync()
            print(f"[configs] {rule}/{topology}: warmup step {i} done", file=sys.stderr,
                  flush=True)
    tr.timer.summary()
    if a.profile_marker and cuda:
        torch.cuda._sleep(1000)
    sync()
    if info.distributed:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    loss = None
    for _ in range(a.steps):
        loss = tr.train_step()
    tr.engine.wait_params()
    sync()
    if info.distributed:
        dist.barrier()
    sync()
    dt = time.perf_counter() - t0
    phases = {k: round(v / a.steps, 3) for k, v in tr.timer.summary().items()}
    if info.distributed:
        t = torch.tensor([dt], dtype=torch.float64, device=info.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
    e = tr.engine
    res = {"dt": dt, "cfg": cfg, "n": n, "phases": phases, "loss": float(loss),
           "params": e.flat.real_numel, "buckets": len(e.flat.buckets),
           "samples_per_item": tr.task.samples_per_item,
           "batched_workers": bool(n > info.world and tr.task.batched_workers
                                   and perf.policy().batched_workers and cuda
                                   and cfg.dtype == "bf16"),
           "replicas_identical": (replicas_identical(e.flat.flat_param)
                                  if info.distributed and topology != "gossip" else None),
           "selection_counts": [int(x) for x in e.sel_counts.tolist()]}
    if cuda:
        res["max_mem_gb"] = round(torch.cuda.max_memory_allocated() / 2 ** 30, 2)
    if topology == "gossip":
        gb = lambda t: round(t.numel() * t.element_size() / 2 ** 30, 2)   # noqa: E731
        res["gossip"] = {
            "gossip_graph": cfg.topology.gossip_graph, "gossip_async": cfg.topology.gossip_async,
            "gossip_exchanged": bool(e.nb_bufs),
            "memory_plan_gib": {
                "params_bf16": gb(e.flat.flat_param), "grads": gb(e.flat.flat_grad),
                "master_fp32": gb(e.master),
                "optimizer_state": round(sum(gb(t) for t in (e.s1, e.s2) if t is not None), 2),
                "neighbour_buffers": round(sum(gb(t) for t in e.nb_bufs), 2),
                "send_buffer": gb(e._send_buf) if e._send_buf is not None else 0.0,
                "n_neighbour_buffers": len(e.nb_bufs)}}
    tr.close()
    del tr, e
    if cuda:
        torch.cuda.empty_cache()
    return res


def main(argv=None):
    a = parse(argv)
    from consensusml_amd.utils.launch import launch_or_check
    world_env = launch_or_check(a.gpus, __file__, tag="configs")
    c = dict(CONFIGS[a.config])
    if a.model:
        c["model"] = a.model
    from consensusml_amd import perf
    from consensusml_amd.parallel.dist import init_distributed
    from consensusml_amd.utils.tuning import configure_miopen
    configure_miopen()
    backend = a.dist_backend if a.dist_backend != "auto" else c.get("backend", "auto")
    if backend == "gloo" and torch.cuda.is_available() and os.environ.get("CML_MLP_GPU") == "1":
        backend = "auto"
    if world_env > 1 and backend == "auto":
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    share = backend == "gloo" and torch.cuda.is_available() and c["dtype"] == "bf16"
    info = init_distributed(backend, device="cuda:0" if share else None, timeout_s=a.timeout,
                            loopback=a.loopback)
    seen = dist.get_world_size() if dist.is_initialized() else 1
    if seen != a.gpus or info.world != a.gpus:
        print(f"[configs] error: --gpus {a.gpus} but the process group has {seen} rank(s)",
              file=sys.stderr)
        sys.exit(2)
    torch.backends.cudnn.benchmark = info.device.type == "cuda"
    main_res = run_config(c, a, info, c["rule"], c["topology"])
    base = None
    if not a.no_baseline:
        base = run_config(c, a, info, "mean", "allreduce")
    cfg = main_res["cfg"]
    n, dt = main_res["n"], main_res["dt"]
    samples = a.steps * cfg.batch_per_worker * n
    ms = dt / a.steps * 1e3
    out = {"config": a.config, "model": cfg.model.name, "rule": cfg.agg.rule,
           "topology": cfg.topology.kind, "n_gpus": info.world, "workers": n, "f": cfg.agg.f,
           "per_worker_batch": cfg.batch_per_worker, "seq_len": cfg.model.seq_len,
           "dtype": cfg.dtype, "optimizer": cfg.optim.name, "params": main_res["params"],
           "bucket_mb": cfg.topology.bucket_mb, "buckets": main_res["buckets"],
           "direct_grads": cfg.topology.direct_grads,
           "samples_per_s": round(samples / dt, 2),
           "tokens_per_s": round(samples * main_res["samples_per_item"] / dt, 1),
           "ms_per_step": round(ms, 3), "phase_ms_per_step": main_res["phases"],
           "loss": main_res["loss"], "data": "synthetic (random-init weights)",
           "steps": a.steps, "warmup": a.warmup,
           "batched_workers": main_res["batched_workers"],
           "allreduce_ms_per_step": None, "agg_overhead_vs_allreduce": None,
           "replicas_identical": main_res["replicas_identical"],
           "selection_counts": main_res["selection_counts"],
           "dist_backend": dist.get_backend() if dist.is_initialized() else None,
           "world_size_seen": seen, "loopback": info.loopback,
           "launcher": ("self" if os.environ.get("CML_BENCH_SELF_LAUNCHED") else
                        "external" if "WORLD_SIZE" in os.environ else "none"),
           "perf_policy": perf.policy().to_dict(), "env_switches": perf.env_switches()}
    if base is not None:
        b_ms = base["dt"] / a.steps * 1e3
        out["allreduce_ms_per_step"] = round(b_ms, 3)
        out["allreduce_samples_per_s"] = round(samples / base["dt"], 2)
        out["agg_overhead_vs_allreduce"] = round((ms - b_ms) / b_ms, 4)
        out["allreduce_phase_ms_per_step"] = base["phases"]
        if base["replicas_identical"] is not None:
            out["allreduce_replicas_identical"] = base["replicas_identical"]
    for k in ("max_mem_gb", "gossip"):
        if k in main_res:
            if k == "gossip":
                out.update(main_res[k])
            else:
                out[k] = main_res[k]
    if info.rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "a") as fh:
                fh.write(line + "\n")
    if info.distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
