"""ConsensusTrainer — the user-facing trainer API (N11).

Mirrors the reference's "trainer returns a named result list" convention: ``runLasso`` returns
``training.set, testing.set, contrast, train.fit, cv.fit, confusionMatrix, test.error,
final.model, nonzero.coef, seed`` (`composite_code/rnotebook/cml_targetaml_seanalysis.Rmd:117-121`)
and ``runSVM`` ``options_string, svm_model, weightsvect, predictions_*, performance_test, ...``
(`...seanalysis.Rmd:189-207`). ``fit`` / ``evaluate`` here return dicts with the same spirit
(snake_case keys): ``final_model, history, confusion_matrix, test_error, tpr, tnr, fdr, for,
selection_counts, seed, options_string``.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional

import torch

from ..config import TrainConfig
from ..models import Task, build_task
from ..parallel.dist import DistInfo, init_distributed
from ..parallel.engine import ConsensusEngine
from ..perf import policy as _P
from ..utils.logging import JsonlLogger, PhaseTimer
from .checkpoint import latest_checkpoint, load_checkpoint, save_checkpoint


class ConsensusTrainer:
    def __init__(self, cfg: TrainConfig, task: Optional[Task] = None,
                 info: Optional[DistInfo] = None):
        self.cfg = cfg
        self.info = info or init_distributed(cfg.backend)
        dev = self.info.device
        dtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[cfg.dtype]
        self.task = task or build_task(cfg.model, dev, dtype, seed=cfg.seed)
        self.engine = ConsensusEngine(self.task.model, cfg, self.info)
        # one data stream per (global) worker id, so a run with R ranks x V virtual workers sees
        # the same batches as a run with 1 rank x R*V virtual workers
        V = self.engine.V
        self.gens = []
        for v in range(V):
            g = torch.Generator(device=dev)
            g.manual_seed(cfg.seed * 1000 + self.info.rank * V + v)
            self.gens.append(g)
        self.gen = self.gens[0]
        # native record loader (csrc/runtime): one disjoint data share per global worker
        self.loaders = []
        if cfg.data_path:
            from ..runtime import DeviceLoader
            shape, fdt, odt = record_spec(cfg, dtype)
            for v in range(V):
                self.loaders.append(DeviceLoader(
                    cfg.data_path, shape, fdt, cfg.batch_per_worker, dev,
                    rank=self.info.rank * V + v, world=self.engine.n, seed=cfg.seed,
                    threads=cfg.loader_threads, out_dtype=odt))
        self.logger = JsonlLogger(cfg.log_path, self.info.rank)
        self.timer = PhaseTimer(dev, enabled=cfg.profile)
        self.history: List[float] = []

    @property
    def model(self) -> torch.nn.Module:
        return self.engine.model

    # ------------------------------------------------------------------ training
    def train_step(self) -> torch.Tensor:
        """One consensus step; returns the mean local loss as a device tensor (no host sync)."""
        e, t = self.engine, self.timer
        self.model.train()
        e.zero_grad()
        if (e.V > 1 and self.task.batched_workers and _P().batched_workers
                and e.device.type == "cuda" and self.cfg.dtype == "bf16"):
            return self._batched_step()
        total = None
        try:
            for v in range(e.V):
                e.bind_worker(v)
                with t.phase("data"):
                    batch = self._worker_batch(v)
                with t.phase("fwd_bwd"):
                    loss = self.task.loss_fn(self.model, batch)
                    loss.backward()
                total = loss.detach() if total is None else total + loss.detach()
        except BaseException:
            # the direct-gradient destination zero_grad() activated is module-global: never
            # leave it active (keyed by id(p), reusable after GC) past a failed step
            e.abort_step()
            raise
        with t.phase("exchange_aggregate_update"):
            e.step()
        return total / e.V

    def _worker_batch(self, v: int):
        if self.loaders:
            x, yb, _ = self.loaders[v].next()
            if x.dim() == 4:
                x = x.contiguous(memory_format=torch.channels_last)
            return x, yb
        return self.task.make_batch(self.cfg.batch_per_worker, self.gens[v])

    def _batched_step(self) -> torch.Tensor:
        """Virtual workers as ONE forward / backward over the V micro-batches (same data as
        the sequential loop: worker v's batch from its own stream), per-worker gradients written
        to the engine's rows by the ops (ConsensusEngine.worker_batch). The loss is the mean over
        all V micro-batches; scaling it by V gives every activation exactly worker v's own
        gradient (equal-sized micro-batches, mean reductions)."""
        e, t = self.engine, self.timer
        with t.phase("data"):
            parts = [self._worker_batch(v) for v in range(e.V)]
            batch = tuple(torch.cat(z) for z in zip(*parts))
        with t.phase("fwd_bwd"):
            with e.worker_batch():
                loss = self.task.loss_fn(self.model, batch)
                (loss * e.V).backward()
        with t.phase("exchange_aggregate_update"):
            e.step()
        return loss.detach()

    def fit(self, steps: Optional[int] = None, log_every: int = 10,
            resume: bool = False) -> Dict[str, object]:
        steps = steps if steps is not None else self.cfg.steps
        if resume and self.cfg.ckpt_dir and latest_checkpoint(self.cfg.ckpt_dir):
            load_checkpoint(self.cfg.ckpt_dir, self.engine, self.gens)
        start = self.engine.step_count
        t0 = time.perf_counter()
        losses = []
        stats_ok = self.engine.topo in ("sharded", "allgather")
        for s in range(start, steps):
            ckpt_now = bool(self.cfg.ckpt_every and self.cfg.ckpt_dir
                            and (s + 1) % self.cfg.ckpt_every == 0)
            log_now = bool(log_every and (s + 1) % log_every == 0)
            # consensus table / log stats of this step. The stats all-reduce is collective, so
            # the decision must be the same on every rank: it depends on the config only, not
            # on logger.enabled (rank 0 alone logs)
            if stats_ok and (ckpt_now or (log_now and bool(self.cfg.log_path))):
                self.engine.record_stats = True
            loss = self.train_step()
            losses.append(loss)
            if log_now:
                lv = float(loss)
                self.logger.log(step=s + 1, loss=lv, phases=self.timer.summary(),
                                **self._log_stats())
            if ckpt_now:
                save_checkpoint(self.cfg.ckpt_dir, self.engine, self.cfg, gens=self.gens,
                                table=self._consensus_table())
        self.engine.wait_params()      # the last step's overlapped parameter all-gather
        if self.info.device.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        hist = [float(l) for l in losses]
        self.history.extend(hist)
        n_done = max(steps - start, 0)
        samples = n_done * self.cfg.batch_per_worker * self.engine.n
        return {
            "final_model": self.model,
            "history": hist,
            "steps": steps,
            "seed": self.cfg.seed,
            "selection_counts": self.engine.sel_counts.cpu().tolist(),
            "last_weights": self.engine.w[: self.engine.n].cpu().tolist(),
            "options_string": f"rule={self.cfg.agg.rule} topology={self.cfg.topology.kind} "
                              f"n={self.engine.n} f={self.cfg.agg.f} optim={self.cfg.optim.name}",
            "samples_per_sec": samples / dt if dt > 0 else float("nan"),
            "wall_s": dt,
        }

    def _log_stats(self) -> Dict[str, object]:
        """Observability fields of a JSONL step record: selection counts and
        aggregation weights of the rule, and -- when the step was recorded -- per-worker gradient
        norms, distances to the aggregate and Krum scores (whole model)."""
        e = self.engine
        out: Dict[str, object] = {"selection_counts": e.sel_counts.cpu().tolist(),
                                  "weights": e.w[: e.n].float().cpu().tolist()}
        st = e.last_stats
        if st is not None and st.get("step") == e.step_count - 1:   # recorded by the last step
            out["worker_grad_norm"] = st["sqnorm"].sum(0).sqrt().tolist()
            out["worker_dist_to_aggregate"] = st["dist2"].sum(0).sqrt().tolist()
            out["aggregate_grad_norm"] = float(st["agg_sqnorm"].sum().sqrt())
            if st.get("scores") is not None:
                out["krum_scores"] = st["scores"].tolist()
        return out

    # ------------------------------------------------------------------ evaluation
    @torch.no_grad()
    def evaluate(self, batches: int = 4, batch_size: Optional[int] = None) -> Dict[str, object]:
        """Loss / accuracy / confusion-derived metrics on fresh synthetic batches."""
        from ..select.metrics import binary_metrics, confusion_matrix
        self.engine.wait_params()
        self.model.eval()
        gen = torch.Generator(device=self.info.device)
        gen.manual_seed(self.cfg.seed + 99991)
        bs = batch_size or self.cfg.batch_per_worker
        ys, ps, losses = [], [], []
        for _ in range(batches):
            x, y = self.task.make_batch(bs, gen)
            out = self.model(x).float()
            losses.append(torch.nn.functional.cross_entropy(out.view(-1, out.shape[-1]),
                                                            y.view(-1)).item())
            ps.append(out.argmax(-1).view(-1))
            ys.append(y.view(-1))
        y = torch.cat(ys).cpu()
        p = torch.cat(ps).cpu()
        res: Dict[str, object] = {"loss": sum(losses) / len(losses),
                                  "accuracy": float((p == y).float().mean()),
                                  "test_error": float((p != y).float().mean())}
        if int(max(y.max(), p.max())) <= 1:
            res["confusion_matrix"] = confusion_matrix(y, p, 2).tolist()
            res.update(binary_metrics(y, p))
        self.model.train()
        return res

    # ------------------------------------------------------------------ checkpoint
    def _consensus_table(self):
        return self.engine.consensus_table() if self.engine.last_stats is not None else None

    def consensus_table(self):
        """Per-parameter x per-worker gradient table of the last recorded step (run a step with
        ``engine.record_stats = True`` first; checkpoints record it automatically)."""
        return self.engine.consensus_table()

    def save(self, root: Optional[str] = None) -> str:
        return save_checkpoint(root or self.cfg.ckpt_dir, self.engine, self.cfg, gens=self.gens,
                               table=self._consensus_table())

    def load(self, path: str) -> dict:
        return load_checkpoint(path, self.engine, self.gens)

    def close(self) -> None:
        self.logger.close()
        self.engine.close()
        for l in self.loaders:
            l.close()


def record_spec(cfg: TrainConfig, dtype: torch.dtype):
    """(feature shape, on-disk dtype, compute dtype) of a model's record files."""
    m = cfg.model
    if m.name == "mlp":
        return (m.in_features,), torch.float32, dtype
    if m.name.startswith("resnet"):
        return (3, m.image_size, m.image_size), torch.float16, dtype
    return (m.seq_len,), torch.int64, None


def write_synthetic_records(cfg: TrainConfig, path: str, n: int, seed: int = 0) -> int:
    """Write ``n`` records of the model's shape drawn from its synthetic generator."""
    import numpy as np
    from ..models import build_task
    from ..runtime import write_records
    task = build_task(cfg.model, torch.device("cpu"), torch.float32, seed=cfg.seed)
    g = torch.Generator().manual_seed(seed)
    x, y = task.make_batch(n, g)
    shape, fdt, _ = record_spec(cfg, torch.float32)
    feats = x.to(fdt).contiguous().numpy().reshape(n, -1)
    return write_records(path, feats, y.numpy().reshape(n, -1)[:, 0])
