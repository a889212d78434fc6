"""Typed configuration for the consensus engine.

The reference has no config system: hyper-parameters, seeds and paths are globals at the top of
each notebook (`composite_code/rnotebook/cml_targetaml_seanalysis.Rmd:370-406`), knitr chunk
options (`...seanalysis.Rmd:10-22`) and literals inside calls (`scripts/model_comp.py:7-9`).
Here one dataclass tree covers model, aggregation rule, topology, optimizer, fault injection and
profiling, with YAML files and ``key.sub=value`` CLI overrides on top.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import yaml

RULES = ("mean", "median", "trimmed_mean", "krum", "multi_krum", "geomed", "bulyan", "centered_clip")
TOPOLOGIES = ("allreduce", "allgather", "sharded", "gossip")
GOSSIP_GRAPHS = ("ring", "exp", "exp_all")
FAULTS = ("none", "sign_flip", "gaussian", "scaled", "zero", "nan", "alie", "ipm")


@dataclass
class AggConfig:
    """Robust aggregation rule and its parameters.

    rule          one of RULES
    f             number of Byzantine workers tolerated (Krum / Multi-Krum / Bulyan)
    trim          number trimmed from each side per coordinate (trimmed mean); ``None`` -> f
    m             number of workers averaged by Multi-Krum; ``None`` -> n - f
    iters, eps    Weiszfeld iterations and distance floor (geometric median)
    tau, clip_iters  radius / iterations of centered clipping
    centered_gram Gram-space rules: the Gram of the rows relative to a medoid worker row, so
                  near-duplicate workers' distances do not cancel (ops.kernels.gram). ONE pass
                  per step, centered at the medoid picked from the previous step's Gram; the
                  first step (and a restore from a checkpoint that has no center) runs an
                  uncentered pass first to pick it
    gram_two_pass every step: uncentered pass -> medoid -> centered pass (+ a second Gram
                  all-reduce in the sharded topology); the round-3 scheme
    """
    rule: str = "mean"
    f: int = 0
    trim: Optional[int] = None
    m: Optional[int] = None
    iters: int = 8
    eps: float = 1e-6
    tol: float = 1e-7
    tau: float = 10.0
    clip_iters: int = 3
    centered_gram: bool = True
    gram_two_pass: bool = False

    def validate(self, n: int) -> None:
        if self.rule not in RULES:
            raise ValueError(f"unknown aggregation rule {self.rule!r}; choose from {RULES}")
        # the HIP kernels keep one worker row per lane of a 64-wide wave; centered clipping adds
        # the previous aggregate as row n
        limit = 63 if self.rule == "centered_clip" else 64
        if n > limit:
            raise ValueError(f"{self.rule} supports at most {limit} workers (n={n})")
        if self.rule in ("krum", "multi_krum") and n > 1 and n <= 2 * self.f:
            # Krum's guarantee needs n >= 2f+3; smaller n runs (nearest-neighbour scoring) but
            # f < n/2 is the hard floor.
            raise ValueError(f"{self.rule} needs n > 2f (n={n}, f={self.f})")
        if self.rule == "bulyan" and n > 1 and n < 4 * self.f + 3:
            raise ValueError(f"bulyan needs n >= 4f+3 (n={n}, f={self.f})")
        b = self.trim if self.trim is not None else self.f
        if self.rule == "trimmed_mean" and 2 * b >= n:
            raise ValueError(f"trimmed_mean needs n > 2*trim (n={n}, trim={b})")


@dataclass
class OptimConfig:
    name: str = "sgd"            # sgd | adam | adamw
    lr: float = 0.1
    momentum: float = 0.9
    nesterov: bool = False
    weight_decay: float = 0.0
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8


@dataclass
class TopologyConfig:
    kind: str = "sharded"        # allreduce | allgather | sharded | gossip
    bucket_mb: float = 64.0      # bucket size in MB of gradient (bf16 on the wire)
    comm_dtype: str = "bf16"     # dtype of exchanged gradients
    overlap: bool = True         # launch bucket collectives during backward
    gossip_graph: str = "ring"   # ring | exp (one rotating peer 2^(t mod log2 N)) | exp_all
    gossip_chunk_mb: float = 256.0   # gossip exchange pipeline chunk (MB of bf16)
    gossip_weights: tuple = (1 / 3, 1 / 3, 1 / 3)   # ring: self, left, right
    gossip_clip: float = 0.0     # 0 disables neighbour-delta clipping
    gossip_async: bool = False   # delayed gossip: exchange overlaps the next step's compute
    early_update: bool = True    # gossip, 1 local worker: per-bucket optimizer step in backward
    param_prefetch: bool = True  # sharded: bf16 parameter all-gather overlaps the next forward
    early_gram: bool = True      # Gram-space rules: per-bucket Gram as each exchange lands
    gram_lag: int = 1            # GPU runs: bucket b's Gram is enqueued on the compute stream at
                                 # the flush of bucket b + gram_lag (its exchange has had one
                                 # bucket of backward to land); the last ones run in step()
    direct_grads: bool = True    # one worker per rank: ops with a per-worker gradient path
                                 # (ops.worker_grads: transformer linears, norms, embeddings) write
                                 # their parameter gradients straight into the flat gradient row
                                 # during backward instead of autograd tensors + the capture copy

    def validate(self) -> None:
        if self.kind not in TOPOLOGIES:
            raise ValueError(f"unknown topology {self.kind!r}; choose from {TOPOLOGIES}")
        if self.gossip_graph not in GOSSIP_GRAPHS:
            raise ValueError(f"unknown gossip graph {self.gossip_graph!r}; choose from "
                             f"{GOSSIP_GRAPHS}")
        if self.gossip_chunk_mb <= 0:
            raise ValueError("gossip_chunk_mb must be positive")


@dataclass
class FaultConfig:
    kind: str = "none"
    ranks: List[int] = field(default_factory=list)   # Byzantine ranks / virtual workers
    scale: float = 10.0
    sigma: float = 1.0
    z: float = 1.0               # ALIE z-score
    start_step: int = 0

    def validate(self) -> None:
        if self.kind not in FAULTS:
            raise ValueError(f"unknown fault {self.kind!r}; choose from {FAULTS}")


@dataclass
class ModelConfig:
    name: str = "mlp"            # mlp | resnet50 | bert_base | llama3_8b | llama_tiny | bert_tiny
    num_classes: int = 1000
    image_size: int = 224
    seq_len: int = 128
    in_features: int = 32
    hidden: int = 64
    extra: Dict[str, Any] = field(default_factory=dict)


@dataclass
class TrainConfig:
    model: ModelConfig = field(default_factory=ModelConfig)
    agg: AggConfig = field(default_factory=AggConfig)
    optim: OptimConfig = field(default_factory=OptimConfig)
    topology: TopologyConfig = field(default_factory=TopologyConfig)
    fault: FaultConfig = field(default_factory=FaultConfig)
    batch_per_worker: int = 32
    virtual_workers: int = 1     # >1: each rank simulates this many workers (micro-batches)
    steps: int = 10
    seed: int = 2019             # the reference's split seed (DEL:159)
    dtype: str = "bf16"
    backend: str = "auto"        # auto | nccl | gloo
    data_path: Optional[str] = None   # record file for the native loader (else synthetic)
    loader_threads: int = 4
    log_path: Optional[str] = None
    ckpt_dir: Optional[str] = None
    ckpt_every: int = 0
    profile: bool = False

    # ------------------------------------------------------------------ io
    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    def to_json(self) -> str:
        return json.dumps(self.to_dict(), sort_keys=True)

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "TrainConfig":
        cfg = cls()
        for k, v in (d or {}).items():
            _set_path(cfg, k, v)
        return cfg

    @classmethod
    def from_yaml(cls, path: str) -> "TrainConfig":
        with open(path) as fh:
            return cls.from_dict(_flatten(yaml.safe_load(fh) or {}))

    def override(self, items: List[str]) -> "TrainConfig":
        """Apply ``a.b=value`` overrides (value parsed as YAML scalar/list)."""
        for it in items:
            if "=" not in it:
                raise ValueError(f"override {it!r} must look like key.sub=value")
            k, v = it.split("=", 1)
            _set_path(self, k, yaml.safe_load(v))
        return self

    def validate(self, n_workers: int) -> "TrainConfig":
        self.agg.validate(n_workers)
        self.topology.validate()
        self.fault.validate()
        return self


def _flatten(d: Dict[str, Any], prefix: str = "") -> Dict[str, Any]:
    out: Dict[str, Any] = {}
    for k, v in d.items():
        key = f"{prefix}{k}"
        if isinstance(v, dict) and k != "extra":
            out.update(_flatten(v, key + "."))
        else:
            out[key] = v
    return out


def _set_path(obj: Any, path: str, value: Any) -> None:
    parts = path.split(".")
    for p in parts[:-1]:
        if not hasattr(obj, p):
            raise KeyError(f"unknown config key {path!r}")
        obj = getattr(obj, p)
    last = parts[-1]
    if not hasattr(obj, last):
        raise KeyError(f"unknown config key {path!r}")
    cur = getattr(obj, last)
    if isinstance(cur, tuple) and isinstance(value, list):
        value = tuple(value)
    if isinstance(cur, float) and isinstance(value, int):
        value = float(value)
    setattr(obj, last, value)


def add_cli(parser: argparse.ArgumentParser) -> argparse.ArgumentParser:
    parser.add_argument("--config", type=str, default=None, help="YAML config file")
    parser.add_argument("--set", nargs="*", default=[], help="overrides key.sub=value")
    return parser


def from_cli(args: argparse.Namespace) -> TrainConfig:
    cfg = TrainConfig.from_yaml(args.config) if args.config else TrainConfig()
    return cfg.override(args.set or [])
