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
aggregation and optimizer update. Per-GPU batch 2560 by default: 288 GB of HBM holds it many
times over (peak ~65 GiB), and throughput still rises with batch. 2560 (not 2048) because the
MFMA-bound 3x3 convs of layers 3 / 4 run 256 x 256 output tiles: at 2048 they are 1568 / 784
tiles = 6.1 / 3.1 rounds of the 256 CUs (7 / 4 launched), at 2560 1960 / 980 = 7.7 / 3.8 rounds
(8 / 4): +1.6-2.2 % samples/s on one box (profiles/r06_07/). 2560 is also the largest batch whose
112 x 112 x 64 stem activations stay under 2^31 elements (int32 element indexing in the stem
kernels).

Communication-visible block (``b256_*`` keys, every N): at batch 2048 the step is ~127 ms of
compute, so at N = 8 the exposed exchange is far below 1 % and "agg overhead vs all-reduce" says
little. The bench therefore also times per-GPU batch 256 (the batch a real 8-GPU DP run uses,
~22 ms of compute per step) with Krum over the sharded exchange vs the mean all-reduce baseline:
``b256_agg_overhead_vs_allreduce`` is the robust-aggregation overhead where communication is
visible. Gradient buckets default to 8 MB (ResNet-50: 7 buckets), so the last all-to-all -- the
one that cannot hide behind backward -- moves ~8 MB instead of 25.

Robust aggregation at one GPU. With one rank there is one worker, so the dp line's Krum is
vacuous there (n = 1, f = 0, nothing exchanged). At N = 1 the bench therefore also runs a
*virtual-worker* block: 8 workers x 256 images on the one GPU (each worker's gradient kept in its
own row, n = 8, f = 2): real Krum (MFMA Gram -> scores -> selection -> fused weighted update)
against the plain mean of the same 8 micro-batch gradients at the same global batch, reported
as ``krum_n8_virtual_*`` keys. At N > 1 the JSON carries ``dist_backend``, ``world_size_seen``,
the exchange + aggregation + update time per step that is NOT hidden behind backward (HIP
events around ``engine.step()``) and a cross-rank bitwise parameter-checksum check
(``replicas_identical``).
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
    ap.add_argument("--batch", type=int, default=2560,
                    help="per-GPU batch (samples/s on MI355X rise with batch, see README; peak "
                         "memory ~65 GiB at 2560 of 288; the shipped MIOpen find-db covers "
                         "256 / 512 / 1024 / 1536 / 2048 / 2560)")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--rule", default="krum")
    ap.add_argument("--f", type=int, default=-1,
                    help="Byzantine tolerance of the dp run (-1: the largest f with n >= 2f+3, "
                         "at least 1 once n >= 4)")
    ap.add_argument("--topology", default="sharded")
    ap.add_argument("--bucket-mb", type=float, default=8.0)
    ap.add_argument("--b256-batch", type=int, default=256,
                    help="per-GPU batch of the communication-visible Krum vs all-reduce block "
                         "(0: off)")
    ap.add_argument("--b256-steps", type=int, default=30)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--no-baseline", action="store_true")
    ap.add_argument("--baseline-steps", type=int, default=-1)
    ap.add_argument("--virtual-workers", type=int, default=-1,
                    help="workers of the virtual-worker Krum block (-1: 8 at N = 1, off at N > 1; "
                         "0: off)")
    ap.add_argument("--virtual-batch", type=int, default=256, help="images per virtual worker")
    ap.add_argument("--virtual-f", type=int, default=2)
    ap.add_argument("--virtual-steps", type=int, default=-1, help="-1: same as --steps")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 (nccl = RCCL; gloo only to rehearse "
                         "several ranks sharing one GPU)")
    ap.add_argument("--loopback", choices=["auto", "on", "off"], default="auto",
                    help="N = 1: run the engine's distributed code path on a 1-rank process group "
                         "(every all-to-all / all-gather / all-reduce goes through RCCL, to this "
                         "rank itself). auto: on with nccl on a GPU")
    ap.add_argument("--timeout", type=float, default=900.0,
                    help="seconds any collective may block before the run fails (non-zero exit)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--conv1x1", choices=["auto", "gemm", "miopen"], default="auto",
                    help="1x1 stride-1 conv forward / data gradient as hipBLASLt GEMMs: per-shape "
                         "measured choice (auto), always, or never (MIOpen)")
    ap.add_argument("--profile-marker", action="store_true",
                    help="launch a spin_kernel between warmup and timed steps (prof_summary --after)")
    ap.add_argument("--no-miopen-find", action="store_true",
                    help="disable MIOpen find mode (torch.backends.cudnn.benchmark) for convs")
    return ap.parse_args()


def default_f(n: int) -> int:
    """Largest f with Krum's n >= 2f + 3, but at least 1 once n >= 4 (n > 2f + 1 keeps one
    nearest neighbour in every score)."""
    if n < 4:
        return 0
    return max(1, (n - 3) // 2)


def param_checksum(flat_param: torch.Tensor) -> torch.Tensor:
    """Exact position-weighted int64 checksum of the parameter bits (equal iff bit-identical,
    up to a negligible collision chance)."""
    bits = flat_param.view(torch.int16).to(torch.int64)
    idx = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) % 65521 + 1
    return torch.stack([(bits * idx).sum(), bits.sum()])


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


class _HostEvent:
    """CPU stand-in for torch.cuda.Event (CPU rehearsals of the launcher / contract)."""

    def __init__(self, **_):
        self.t = 0.0

    def record(self):
        self.t = time.perf_counter()

    def elapsed_time(self, other) -> float:
        return (other.t - self.t) * 1e3


def run(args, rule: str, topology: str, steps: int, warmup: int, info, *, V: int = 1,
        batch: int = 0, f: int = -1):
    from consensusml_amd.parallel.dist import barrier
    from consensusml_amd import TrainConfig
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    batch = batch or args.batch
    n = info.world * V
    cfg = TrainConfig()
    cfg.model.name = args.model
    cfg.model.image_size = args.image_size
    cfg.batch_per_worker = batch
    cfg.virtual_workers = V
    cfg.dtype = "bf16"
    cfg.agg.rule = rule
    cfg.agg.f = f if f >= 0 else (args.f if args.f >= 0 else default_f(n))
    if rule == "mean":
        cfg.agg.f = 0
    cfg.topology.kind = topology
    cfg.topology.bucket_mb = args.bucket_mb
    cfg.topology.overlap = not args.no_overlap
    cfg.optim.name = "sgd"
    cfg.optim.lr = 0.1
    cfg.optim.momentum = 0.9
    cfg.optim.weight_decay = 5e-5
    tr = ConsensusTrainer(cfg, info=info)
    dev = info.device
    # pre-generate a few synthetic batches per worker (data generation is not part of the step)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + info.rank)
    batches = [[tr.task.make_batch(batch, gen) for _ in range(V)] for _ in range(2)]
    model, eng = tr.model, tr.engine
    tag = f"{rule}/{topology}" + (f" V={V}x{batch}" if V > 1 else "")
    ev = []

    def step(i, timed=False):
        eng.zero_grad()
        loss = None
        for v in range(V):
            if V > 1:
                eng.bind_worker(v)
            lv = tr.task.loss_fn(model, batches[i % len(batches)][v])
            lv.backward()
            loss = lv.detach() if loss is None else loss + lv.detach()
        if timed:
            Ev = torch.cuda.Event if dev.type == "cuda" else _HostEvent
            e0 = Ev(enable_timing=True)
            e1 = Ev(enable_timing=True)
            e0.record()
            eng.step()
            e1.record()
            ev.append((e0, e1))
        else:
            eng.step()
        return loss / V

    tw = time.perf_counter()
    for i in range(max(warmup, 1 if torch.backends.cudnn.benchmark else 0)):
        step(i)
        if info.rank == 0:   # progress: a cold MIOpen find for new conv shapes can take minutes
            _sync()
            print(f"[bench] {tag}: warmup step {i} done at {time.perf_counter() - tw:.1f}s",
                  file=sys.stderr, flush=True)
    _sync()
    if info.rank == 0:
        print(f"[bench] {tag}: warmup {time.perf_counter() - tw:.1f}s", file=sys.stderr,
              flush=True)
    if args.profile_marker:
        torch.cuda._sleep(1000)
    barrier()
    _sync()
    t0 = time.perf_counter()
    for i in range(steps):
        loss = step(i, timed=True)
    eng.wait_params()             # the last step's overlapped parameter all-gather
    _sync()
    barrier()
    _sync()
    dt = time.perf_counter() - t0
    step_ms = sum(a.elapsed_time(b) for a, b in ev) / max(len(ev), 1)
    if info.distributed:
        t = torch.tensor([dt, step_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, step_ms = float(t[0].item()), float(t[1].item())
    finite = bool(torch.isfinite(loss).item())
    res = {"dt": dt, "f": cfg.agg.f, "n": n, "loss": float(loss.item()), "finite": finite,
           "params": eng.flat.real_numel, "buckets": len(eng.flat.buckets),
           "engine_step_ms": step_ms, "early_grams": eng.early_grams,
           "steps_run": eng.step_count,
           "selected": int((eng.w[: eng.n] > 0).sum().item()),
           "sel_counts": [int(c) for c in eng.sel_counts.tolist()]}
    if info.distributed:
        # cross-rank check: every replica must hold bit-identical parameters after the run
        cs = param_checksum(eng.flat.flat_param)
        hi, lo = cs.clone(), cs.clone()
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        res["replicas_identical"] = bool(torch.equal(hi, lo))
        res["world_size_seen"] = dist.get_world_size()
        res["dist_backend"] = dist.get_backend()
    tr.close()
    del tr, eng, model, batches
    torch.cuda.empty_cache()
    return res


def self_launch(n: int) -> int:
    """``--gpus N`` without a launcher: N ranks of this script (consensusml_amd.utils.launch)."""
    from consensusml_amd.utils.launch import self_launch as _launch
    return _launch(n, __file__)


def main():
    # CML_TRACEBACK_AFTER=S: dump every thread's Python stack to stderr every S seconds (finds
    # where a rank waits when a multi-rank run stops making progress)
    if os.environ.get("CML_TRACEBACK_AFTER"):
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["CML_TRACEBACK_AFTER"]), repeat=True)
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(self_launch(args.gpus))
    world_env = int(world_env or "1")
    if world_env != args.gpus:
        print(f"[bench] error: --gpus {args.gpus} but WORLD_SIZE={world_env}", file=sys.stderr)
        sys.exit(2)
    from consensusml_amd import perf
    perf.set_policy(perf.policy().replace(conv1x1_gemm=args.conv1x1))
    if not args.no_miopen_find:
        from consensusml_amd.utils.tuning import configure_miopen
        configure_miopen()
    from consensusml_amd.parallel.dist import init_distributed
    loopback = world_env == 1 and (args.loopback == "on" or (
        args.loopback == "auto" and args.dist_backend == "nccl" and torch.cuda.is_available()))
    backend = args.dist_backend if (world_env > 1 or loopback) else "auto"
    share = args.dist_backend == "gloo" and torch.cuda.is_available()
    info = init_distributed(backend, device="cuda:0" if share else None,
                            timeout_s=args.timeout, loopback=loopback)
    seen = dist.get_world_size() if dist.is_initialized() else 1
    if seen != args.gpus or info.world != args.gpus:
        print(f"[bench] error: --gpus {args.gpus} but the process group has {seen} rank(s)",
              file=sys.stderr)
        sys.exit(2)
    if os.environ.get("CML_BENCH_FAIL_RANK") == str(info.rank):   # launcher tests
        print(f"[bench] rank {info.rank}: injected failure", file=sys.stderr, flush=True)
        os._exit(7)
    # MIOpen find mode: conv solvers are benchmarked on first use of each shape (untimed: the
    # warmup steps, plus one tuning step when --warmup 0) and cached for the run.
    torch.backends.cudnn.benchmark = not args.no_miopen_find
    n = info.world
    main_res = run(args, args.rule, args.topology, args.steps, args.warmup, info)
    ms = main_res["dt"] / args.steps * 1e3
    value = n * args.batch * args.steps / main_res["dt"]
    overhead = None
    base = None
    if not args.no_baseline:
        bsteps = args.baseline_steps if args.baseline_steps > 0 else args.steps
        base = run(args, "mean", "allreduce", bsteps, args.warmup, info)
        base["ms"] = base["dt"] / bsteps * 1e3
        overhead = (ms - base["ms"]) / base["ms"]
    V = args.virtual_workers if args.virtual_workers >= 0 else (8 if n == 1 else 0)
    virt = {}
    if V > 1:
        vsteps = args.virtual_steps if args.virtual_steps > 0 else args.steps
        vb = args.virtual_batch
        kr = run(args, "krum", "sharded", vsteps, args.warmup, info, V=V, batch=vb,
                 f=args.virtual_f)
        mn = run(args, "mean", "sharded", vsteps, args.warmup, info, V=V, batch=vb, f=0)
        k_ms = kr["dt"] / vsteps * 1e3
        m_ms = mn["dt"] / vsteps * 1e3
        tag = f"krum_n{kr['n']}_virtual"
        virt = {
            f"{tag}_samples_per_s": round(n * V * vb * vsteps / kr["dt"], 2),
            f"{tag}_ms_per_step": round(k_ms, 3),
            f"{tag}_mean_ms_per_step": round(m_ms, 3),
            f"{tag}_overhead": round((k_ms - m_ms) / m_ms, 4),
            f"{tag}_engine_step_ms": round(kr["engine_step_ms"], 3),
            f"{tag}_mean_engine_step_ms": round(mn["engine_step_ms"], 3),
            f"{tag}_config": {"workers": kr["n"], "f": kr["f"], "per_worker_batch": vb,
                              "global_batch": n * V * vb, "rule": "krum",
                              "baseline": "mean of the same worker rows (same engine, same "
                                          "fused SGD)",
                              "selected_last_step": kr["selected"],
                              "selection_counts": kr["sel_counts"]},
            f"{tag}_loss_finite": kr["finite"] and mn["finite"],
        }
    small = {}
    if args.b256_batch > 0 and args.b256_batch != args.batch:
        sb = args.b256_batch
        ks = run(args, args.rule, args.topology, args.b256_steps, args.warmup, info, batch=sb)
        ar = run(args, "mean", "allreduce", args.b256_steps, args.warmup, info, batch=sb)
        k_ms = ks["dt"] / args.b256_steps * 1e3
        a_ms = ar["dt"] / args.b256_steps * 1e3
        small = {
            "b256_samples_per_s": round(n * sb * args.b256_steps / ks["dt"], 2),
            "b256_ms_per_step": round(k_ms, 3),
            "b256_allreduce_samples_per_s": round(n * sb * args.b256_steps / ar["dt"], 2),
            "b256_allreduce_ms_per_step": round(a_ms, 3),
            "b256_agg_overhead_vs_allreduce": round((k_ms - a_ms) / a_ms, 4),
            "b256_engine_step_ms": round(ks["engine_step_ms"], 3),
            "b256_allreduce_engine_step_ms": round(ar["engine_step_ms"], 3),
            "b256_config": {"per_gpu_batch": sb, "global_batch": n * sb, "rule": args.rule,
                            "f": ks["f"], "topology": args.topology, "buckets": ks["buckets"],
                            "steps": args.b256_steps,
                            "early_grams_per_step": round(ks["early_grams"] /
                                                          max(ks["steps_run"], 1), 2)},
            "b256_loss_finite": ks["finite"] and ar["finite"],
        }
        if info.distributed:
            small["b256_replicas_identical"] = ks["replicas_identical"] and \
                ar["replicas_identical"]
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
            "config": {"model": args.model, "global_batch": n * args.batch, "seq_len": None,
                       "image_size": args.image_size, "per_gpu_batch": args.batch,
                       "parallelism": f"dp{n}", "rule": args.rule, "f": main_res["f"],
                       "topology": args.topology, "optimizer": "sgd-momentum (fused HIP)",
                       "conv1x1": args.conv1x1,
                       "params": main_res["params"], "buckets": main_res["buckets"]},
            "allreduce_ms_per_step": None if base is None else round(base["ms"], 3),
            "agg_overhead_vs_allreduce": None if overhead is None else round(overhead, 4),
            "engine_step_ms": round(main_res["engine_step_ms"], 3),
            "allreduce_engine_step_ms": None if base is None else round(base["engine_step_ms"], 3),
            "loss_finite": main_res["finite"],
            "peak_mem_gib": (round(torch.cuda.max_memory_allocated() / 2**30, 1)
                             if torch.cuda.is_available() else None),
            # every kernel / fusion switch in force (consensusml_amd.perf.PerfPolicy)
            "perf_policy": perf.policy().to_dict(),
            # CML_* overrides of the native launchers' switches (CML_CONV3P, CML_CONV_GEMM2, ...)
            "env_switches": perf.env_switches(),
        }
        if info.distributed:
            out["dist_backend"] = main_res["dist_backend"]
            out["world_size_seen"] = main_res["world_size_seen"]
            out["replicas_identical"] = main_res["replicas_identical"] and (
                base is None or base["replicas_identical"])
        else:
            out["dist_backend"] = None
            out["world_size_seen"] = 1
        out["selection"] = {"n": main_res["n"], "f": main_res["f"],
                            "selected_last_step": main_res["selected"],
                            "selection_counts": main_res["sel_counts"]}
        out["loopback"] = info.loopback
        out["launcher"] = ("self" if os.environ.get("CML_BENCH_SELF_LAUNCHED") else
                           "external" if "WORLD_SIZE" in os.environ else "none")
        out.update(virt)
        out.update(small)
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as fh:
                fh.write(line + "\n")
    if info.distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
