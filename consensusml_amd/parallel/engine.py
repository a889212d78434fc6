"""Consensus data-parallel engine: exchange topologies x robust rules x fused optimizer (N02-N09).

Per step:  zero grads -> forward/backward (autograd accumulates into the flat gradient buffer;
bucket collectives launch from post-accumulate hooks while backward runs) -> fault injection ->
exchange -> robust aggregation fused with the optimizer update -> parameter all-gather.

Topologies:
  allreduce  baseline DDP: RCCL all-reduce(sum) of bf16 buckets, fused update of the full vector.
  allgather  topology A: every rank all-gathers all N gradients ([N, L] per bucket) and runs the
             robust rule on everything (identical, deterministic result on every rank).
  sharded    topology B ("robust ZeRO"): all-to-all so rank r holds coordinate shard r of every
             worker ([N, L/N] per bucket), robust rule + optimizer on the shard only (fp32 master
             and optimizer state are sharded 1/N), then an in-place all-gather of the bf16
             parameter shards. Gram-space rules (Krum, Multi-Krum, Weiszfeld, centered
             clipping, Bulyan's selection) all-reduce the [n, n] fp64 partial Gram (<= 32 KB)
             so every rank derives identical weights. Traffic ~= one ring all-reduce, spread over
             all 7 xGMI links by the all-to-all.
  gossip     topology C: local fused step, then an exchange of bf16 parameters with this step's
             neighbours (grouped send/recv, chunked so exchange of chunk k+1 overlaps mixing of
             chunk k) and a fused, optionally clipped, k-neighbour mixing kernel. Graphs
             (topology.gossip_graph): ring (r +- 1, 2 of the 7 xGMI links); exp (one-peer
             exponential graph: at step t send to r + 2^(t mod tau), receive from r - 2^(t mod
             tau), x <- (x + nb) / 2; exact averaging after tau = ceil(log2 N) steps when N is a
             power of two, half the ring's bytes per step, ONE receive buffer); exp_all (every
             r +- 2^i at once: 5 distinct peers at N = 8, uniform weights 1 / (k + 1)).

Workers = ranks x virtual_workers (micro-batches whose gradients are kept separately), so the
robust rules can be exercised at n = 8 on a single GPU.
"""
from __future__ import annotations

import contextlib
import math

import numpy as np
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..config import TrainConfig
from ..ops import kernels as K
from ..ops import worker_grads as WG
from ..perf import policy as _P
from ..ops.native import lib
from .dist import DistInfo
from .faults import COLLUSION, apply_faults
from .flat import Bucket, FlatModel


GRAM_RULES = ("krum", "multi_krum", "geomed", "centered_clip", "bulyan")


def gossip_peers(graph: str, N: int, r: int, t: int, ring_weights=(1 / 3, 1 / 3, 1 / 3)):
    """(send-to, recv-from, mixing weights, self weight) of rank r at gossip step t.

    ring     r -+ 1 with ``ring_weights`` = (self, left, right)
    exp      one rotating peer: send to r + 2^(t mod tau), receive from r - 2^(t mod tau),
             x <- (x + nb) / 2, tau = ceil(log2 N)
    exp_all  every distinct r +- 2^i (i < tau) at once, uniform weights 1 / (k + 1)
    """
    tau = max(1, (N - 1).bit_length())          # ceil(log2 N)
    if graph == "ring":
        w0, w1, w2 = ring_weights
        left, right = (r - 1) % N, (r + 1) % N
        return [left, right], [left, right], [w1, w2], w0
    if graph == "exp":
        s = 1 << (t % tau)
        return [(r + s) % N], [(r - s) % N], [0.5], 0.5
    peers = []
    for i in range(tau):
        for q in ((r + (1 << i)) % N, (r - (1 << i)) % N):
            if q != r and q not in peers:
                peers.append(q)
    w = 1.0 / (len(peers) + 1)
    return peers, peers, [w] * len(peers), w


def max_gossip_peers(graph: str, N: int) -> int:
    """Largest number of neighbour buffers one mixing step reads, over every rank and step
    (exp_all: 2 ceil(log2 N) - 1 at N = 2^k, e.g. 5 at N = 8 and 9 at N = 32)."""
    tau = max(1, (N - 1).bit_length())
    return max(len(gossip_peers(graph, N, r, t)[1]) for r in range(N) for t in range(tau))


class _EventWork:
    """A work-like handle (``wait()``) for device work enqueued on a side stream: the waiting
    stream (the caller's current stream) waits for an event recorded now on ``stream``."""

    def __init__(self, stream: torch.cuda.Stream):
        self.ev = torch.cuda.Event()
        self.ev.record(stream)

    def wait(self) -> None:
        torch.cuda.current_stream().wait_event(self.ev)


class ConsensusEngine:
    def __init__(self, model: torch.nn.Module, cfg: TrainConfig, info: DistInfo):
        self.cfg = cfg
        self.info = info
        self.N = info.world
        self.V = max(1, cfg.virtual_workers)
        self.n = self.N * self.V
        cfg.validate(self.n)
        self.topo = cfg.topology.kind
        self.rule = cfg.agg.rule
        if self.topo == "allreduce" and self.rule != "mean":
            raise ValueError("the allreduce topology only implements the mean rule")
        pdtype = next(p for p in model.parameters() if p.requires_grad).dtype
        self.flat = FlatModel(model, self.N, cfg.topology.bucket_mb, grad_rows=self.V,
                              param_dtype=pdtype)
        self.device = self.flat.device
        self.rank = info.rank
        self.group_active = info.distributed
        dev = self.device
        fl = self.flat
        if self.group_active:   # identical starting point on every replica
            dist.broadcast(fl.flat_param, src=0)

        # -------------------------------------------------- optimizer state (fp32)
        if self.topo == "sharded":
            self.master = fl.gather_shard_vector(fl.flat_param, self.rank).float().contiguous()
        else:
            self.master = fl.flat_param.float().clone()
        self.state_len = self.master.numel()
        oname = cfg.optim.name
        self.s1 = torch.zeros_like(self.master) if (oname != "sgd" or cfg.optim.momentum) else None
        self.s2 = torch.zeros_like(self.master) if oname in ("adam", "adamw") else None
        self.step_count = 0

        # -------------------------------------------------- exchange buffers
        extra = 1 if self.rule == "centered_clip" else 0
        self.rows_total = self.n + extra
        self.recv: List[torch.Tensor] = []
        if self.topo == "sharded":
            for b in fl.buckets:
                self.recv.append(torch.zeros(self.rows_total, b.shard, dtype=fl.dtype, device=dev))
        elif self.topo == "allgather":
            for b in fl.buckets:
                self.recv.append(torch.zeros(self.rows_total, b.length, dtype=fl.dtype, device=dev))
        self.nb_bufs: List[torch.Tensor] = []
        if self.topo == "gossip" and self.group_active:
            self._setup_gossip()
        self._gossip_reqs = None
        self._send_buf = None
        self._gossip_restored = False   # neighbour buffers restored from a checkpoint
        # -------------------------------------------------- rule buffers
        self.G = torch.zeros(self.rows_total, self.rows_total, dtype=torch.float64, device=dev)
        self.w = torch.full((self.rows_total,), 1.0 / self.n, dtype=torch.float32, device=dev)
        if extra:
            self.w[-1] = 0.0
        self.scores = torch.zeros(self.n, dtype=torch.float64, device=dev)
        self.sel = torch.zeros(self.n + 1, dtype=torch.int32, device=dev)
        self.sel_counts = torch.zeros(self.n, dtype=torch.float64, device=dev)
        # [centered-Gram row, non-finite rows of the previous pass] (weights.hip guard state)
        self.center = torch.zeros(2, dtype=torch.int32, device=dev)
        self.have_center = False    # self.center holds a medoid from an earlier step
        self.gout = None
        if self.rule == "centered_clip":
            self.gout = torch.zeros(self.state_len, dtype=torch.float32, device=dev)

        # -------------------------------------------------- gradient capture + overlap hooks
        # Copy-on-ready: autograd produces fresh .grad tensors; when every parameter of a bucket
        # has its gradient, ONE multi-tensor copy moves them into that bucket of the flat buffer
        # (2 passes instead of zero + accumulate-add's 4, a few launches instead of one per
        # parameter) and, with overlap on, the bucket's collective launches right away while
        # backward keeps running.
        self._pending: Dict[int, object] = {}
        self._ready: Dict[int, List[int]] = {b.index: [] for b in fl.buckets}
        self._flushed: set = set()
        self._in_worker_batch = False
        # TopologyConfig.direct_grads: a one-worker gradient destination (ops.worker_grads) is
        # active from zero_grad() to step(), so the ops with a per-worker gradient path write
        # straight into the flat row; their AccumulateGrad hooks still fire (with no gradient)
        # in autograd order and drive the bucket flushes as before
        self.direct_grads = bool(getattr(cfg.topology, "direct_grads", False) and self.V == 1
                                 and self.device.type == "cuda")
        self._direct_wg = None
        self._direct_prev = None
        self._hooks = []
        self.overlap = bool(cfg.topology.overlap and self.V == 1 and self.group_active
                            and self.topo in ("allreduce", "allgather", "sharded")
                            and cfg.fault.kind not in COLLUSION)
        fl.release_grads(0)
        for i, p in enumerate(fl.params):
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
        self.timings: Dict[str, float] = {}
        # Gossip with one local worker: the local optimizer step needs nothing from other ranks,
        # so each bucket's fused AdamW / SGD runs on a side stream as soon as backward has
        # produced that bucket's gradients (the memory-bound update overlaps the rest of the
        # backward's GEMMs); step() then only waits for it and does the neighbour exchange. A
        # parameter's value is not read again once its gradient exists (its last use in backward
        # produced that gradient), so updating it early is exact.
        self.early_update = (self.topo == "gossip" and self.V == 1 and dev.type == "cuda"
                             and cfg.fault.kind not in COLLUSION
                             and cfg.topology.early_update)
        self._updated: set = set()
        self._opt_stream = torch.cuda.Stream(device=dev) if self.early_update else None
        # Sharded topology: the bf16 parameter all-gather of each bucket is not waited for at the
        # end of step(); the next forward waits per top-level module (forward pre-hooks) for the
        # buckets holding that module's parameters, so the all-gathers of later layers overlap
        # the forward of earlier ones. The all-gathers are launched earliest-layers-first. Which
        # top-level children are actually called as modules (their params are only read inside
        # their own forward) is learned on the first step, which waits for everything up front.
        self._ag_works: Dict[int, object] = {}
        # Delayed gossip on the GPU: the end-of-step mix runs on a side stream bucket by bucket
        # (earliest layers first) and the next forward waits per module for its buckets through
        # the same hooks, so the mix overlaps the forward instead of preceding it
        self._mix_stream = (torch.cuda.Stream(device=dev)
                            if (self.topo == "gossip" and cfg.topology.gossip_async
                                and dev.type == "cuda" and self.group_active) else None)
        self.param_prefetch = bool(cfg.topology.param_prefetch and self.group_active
                                   and (self.topo == "sharded" or self._mix_stream is not None))
        self._prefetch_hooks = []
        if self.param_prefetch:
            self._setup_prefetch()
        # Per-bucket Gram partials (Gram-space rules, sharded / allgather across ranks): slot b
        # holds bucket b's local X X^T. A slot is filled as soon as that bucket's exchange has
        # landed -- polled from the gradient hooks while backward still runs -- and step() sums
        # the slots in bucket order, so the result does not depend on when each was computed.
        self.early_gram = bool(cfg.topology.early_gram and self.rule in GRAM_RULES
                               and self.group_active
                               and self.topo in ("sharded", "allgather"))
        self.Gb = (torch.zeros(len(fl.buckets), self.rows_total, self.rows_total,
                               dtype=torch.float64, device=dev) if self.early_gram else None)
        self._gram_done: set = set()
        self.early_grams = 0       # bucket Grams computed before step() (all steps)
        self._gram_eager = False   # tests: wait for each exchange in its hook (forces the path)
        # GPU ordering of the early Grams, no host polling (a host-side is_completed() poll
        # sees nothing finished: the host runs ahead of the GPU). Bucket b's Gram is enqueued on
        # the compute stream at the flush of bucket b + gram_lag, behind a device-side wait for
        # b's collective -- by then one bucket of backward has run since that collective was
        # issued, so the wait is normally already satisfied, and the small Gram kernel slots in
        # between backward kernels. (A side stream waiting on each collective measured 1.5 ms /
        # step SLOWER at batch 256: the extra stream's waits share hardware queues with the
        # compute stream, profiles/r05_02/bench.json.) CPU / gloo runs keep the polled form.
        self._gram_queue: List[Bucket] = []
        self._gram_arg_cache: Dict[int, tuple] = {}
        self._gram_nblk: Dict[int, int] = {}
        self._fast_gram_ok: Optional[bool] = None
        # One rank only: at N > 1 a device-side wait on a collective that has not
        # landed would hold back every later backward kernel, and no N > 1 run has measured it;
        # there the Grams use the polled form (at N = 8 a rank's shard Gram is ~10 us at step())
        self._gram_ordered = self.early_gram and dev.type == "cuda" and self.N == 1
        self.gram_lag = max(0, int(cfg.topology.gram_lag))
        # training-side consensus table (SURVEY.md §5.4 b): when set, the next step() records
        # per-worker / per-parameter gradient statistics (consensus_table())
        self.record_stats = False
        self.last_stats: Optional[dict] = None

    # ================================================================ public API
    @property
    def model(self) -> torch.nn.Module:
        return self.flat.model

    def zero_grad(self) -> None:
        """Start a step. Gradient rows are fully overwritten by the copy-on-ready hooks (missing
        gradients are zero-filled at flush), so no memset is needed."""
        for p in self.flat.params:
            p.grad = None
        for v in self._ready.values():
            v.clear()
        self._flushed.clear()
        self._pending.clear()
        self._gram_done.clear()
        self._gram_queue.clear()
        self.flat.grad_row = 0
        if self.direct_grads:
            self._end_direct()
            views = self.flat.worker_views()
            self._direct_wg = WG.WorkerGrads(
                1, {id(p): views[i] for i, p in enumerate(self.flat.params)})
            self._direct_prev = WG.activate(self._direct_wg)

    def abort_step(self) -> None:
        """Undo zero_grad()'s per-step state after a failed forward / backward: deactivate the
        direct-gradient destination (module-global) and drop the half-filled bucket state."""
        self._end_direct()
        for v in self._ready.values():
            v.clear()
        self._flushed.clear()

    def _end_direct(self) -> None:
        if self._direct_wg is not None:
            if WG.current() is self._direct_wg:
                WG.activate(self._direct_prev)
            self._direct_wg = self._direct_prev = None

    def bind_worker(self, v: int) -> None:
        """Route the next backward's gradients into virtual-worker row v."""
        if v != self.flat.grad_row:
            self._flush_row()
        self.flat.grad_row = v

    @contextlib.contextmanager
    def worker_batch(self):
        """Batched virtual workers (ops.worker_grads): run the V micro-batches as ONE forward /
        backward inside this context. The parameter-owning ops write worker v's gradient into
        row v of the flat gradient buffer and hand autograd no parameter gradient, so the
        copy-on-ready hooks stay idle; parameters no op produced a gradient for get zero rows.
        Only valid for models without cross-sample coupling (Task.batched_workers)."""
        fl = self.flat
        views = fl.worker_views()
        wg = WG.WorkerGrads(self.V, {id(p): views[i] for i, p in enumerate(fl.params)})
        prev = WG.activate(wg)
        self._in_worker_batch = True
        try:
            yield wg
        finally:
            WG.activate(prev)
            self._in_worker_batch = False
        for i, p in enumerate(fl.params):
            if p.grad is not None:
                raise RuntimeError(
                    f"parameter {fl.param_names()[i]} got an autograd gradient inside "
                    "worker_batch(): its op has no per-worker gradient path")
            if id(p) not in wg.touched:
                views[i].zero_()
        self._flushed = {b.index for b in fl.buckets}
        fl.grad_row = self.V - 1

    # ================================================================ parameter prefetch
    def _setup_prefetch(self) -> None:
        """Forward pre-hooks per unit: the top-level children, except that a container that is
        never called (ModuleList / ModuleDict, e.g. a transformer's layer stack) contributes its
        children (one unit per block)."""
        fl = self.flat
        root = fl.model
        pid = {id(p): i for i, p in enumerate(fl.params)}
        units = []
        for name, child in root.named_children():
            if isinstance(child, (torch.nn.ModuleList, torch.nn.ModuleDict)):
                units += [(f"{name}.{n2}", c2) for n2, c2 in child.named_children()]
            else:
                units.append((name, child))
        covered = {id(p) for _, u in units for p in u.parameters()}
        self._root_buckets = {fl.bucket_of[pid[id(p)]] for p in root.parameters()
                              if id(p) in pid and id(p) not in covered}
        self._child_buckets: Dict[str, set] = {}
        for name, child in units:
            self._child_buckets[name] = {fl.bucket_of[pid[id(p)]] for p in child.parameters()
                                         if id(p) in pid}
            self._prefetch_hooks.append(child.register_forward_pre_hook(
                self._make_child_pre(name)))
        self._prefetch_hooks.append(root.register_forward_pre_hook(self._root_pre))
        self._invoked: set = set()
        self._learned = False

    def _wait_ag(self, bi: int) -> None:
        w = self._ag_works.pop(bi, None)
        if w is not None:
            w.wait()

    def wait_params(self) -> None:
        """Complete every in-flight parameter all-gather (before reading parameters outside a
        forward, e.g. a checkpoint or an evaluation of submodules)."""
        for bi in list(self._ag_works):
            self._wait_ag(bi)

    def _root_pre(self, _mod, _inp):
        if not self._ag_works:
            return
        if not self._learned:
            self.wait_params()
            return
        need = set(self._root_buckets)
        for name, bks in self._child_buckets.items():
            if name not in self._invoked:
                need |= bks
        for bi in need:
            self._wait_ag(bi)

    def _make_child_pre(self, name: str):
        def pre(_mod, _inp):
            # learn only from training forwards (evaluate() / no-grad forwards of a child may
            # differ from how the training forward reads its parameters)
            if not self._learned and self.flat.model.training and torch.is_grad_enabled():
                self._invoked.add(name)
            for bi in self._child_buckets[name]:
                self._wait_ag(bi)
        return pre

    def step(self) -> None:
        """Exchange, aggregate and update (call after all backward passes of the step)."""
        fl = self.flat
        self._end_direct()
        if self.param_prefetch:
            self.wait_params()          # params no forward touched
            if self._invoked:
                self._learned = True
        self._flush_row()
        if self.early_update:
            for b in fl.buckets:       # buckets whose gradients were never all produced
                if b.index not in self._updated:
                    if self.cfg.fault.kind != "none":
                        apply_faults(fl.flat_grad, self.cfg.fault, self.rank, self.step_count,
                                     self.group_active, self.cfg.seed + self.step_count,
                                     cols=slice(b.offset, b.offset + b.length))
                    self._bucket_update(b)
            torch.cuda.current_stream(self.device).wait_stream(self._opt_stream)
        elif not self.overlap or self.cfg.fault.kind in COLLUSION:
            apply_faults(fl.flat_grad, self.cfg.fault, self.rank, self.step_count,
                         self.group_active, self.cfg.seed + self.step_count)
        for b in fl.buckets:
            if b.index not in self._pending:
                self._launch_bucket(b, inject=False)
        if self.topo == "allreduce":
            self._step_allreduce()
        elif self.topo == "allgather":
            self._step_allgather()
        elif self.topo == "sharded":
            self._step_sharded()
        else:
            self._step_gossip()
        self._pending.clear()
        self._flushed.clear()
        self._updated.clear()
        self.step_count += 1

    # ================================================================ hooks / launches
    def _make_hook(self, i: int):
        b = self.flat.buckets[self.flat.bucket_of[i]]
        need = len(b.params)

        def hook(_p):
            if self._in_worker_batch:   # autograd runs the hook even for a None gradient
                return
            lst = self._ready[b.index]
            lst.append(i)
            if len(lst) == need:
                self._flush(b, complete=True)
        return hook

    def _flush(self, b: Bucket, complete: bool) -> None:
        """Copy the ready gradients of bucket b into the current row; zero-fill the rest."""
        fl = self.flat
        views = fl.grad_views(fl.grad_row)
        lst = self._ready[b.index]
        if lst:
            # direct gradients (no autograd tensor) are already in the row; a parameter whose
            # hook fired without a gradient and without a direct write gets a zero row
            wg = self._direct_wg
            cp = []
            for i in lst:
                p = fl.params[i]
                if p.grad is not None:
                    if wg is not None and id(p) in wg.touched:
                        # a direct write AND an autograd gradient (a tied weight with one use on
                        # the direct path): add, never overwrite the direct contribution
                        views[i].add_(p.grad.view_as(views[i]))
                    else:
                        cp.append(i)
                elif wg is None or id(p) not in wg.touched:
                    views[i].zero_()
            dst = [views[i] for i in cp]
            src = [fl.params[i].grad for i in cp]
            # copy-on-ready through the HIP multi-tensor copy (PerfPolicy.multi_copy)
            if not dst:
                pass
            elif dst[0].is_cuda and _P().multi_copy:
                # one HIP launch per 32 tensors at ~HBM speed (csrc/kernels/multi_copy.hip)
                rest = lib().multi_copy(dst, src)
                if rest:
                    torch._foreach_copy_([dst[j] for j in rest], [src[j] for j in rest])
            else:
                torch._foreach_copy_(dst, src)
            for i in lst:
                fl.params[i].grad = None
        if not complete:
            got = set(lst)
            for i in b.params:
                if i not in got:
                    views[i].zero_()
        lst.clear()
        self._flushed.add(b.index)
        if self.overlap and b.index not in self._pending:
            self._launch_bucket(b, inject=True)
            if self.early_gram:
                if self._gram_ordered:
                    self._gram_queue.append(b)
                    while len(self._gram_queue) > self.gram_lag:
                        self._bucket_gram(self._gram_queue.pop(0))
                        self.early_grams += 1
                else:
                    self._poll_grams()
        if self.early_update and complete:
            self._early_update(b)

    def _early_update(self, b: Bucket) -> None:
        """Gossip, V == 1: this bucket's local optimizer step on the side stream."""
        fl = self.flat
        if self.cfg.fault.kind != "none":
            apply_faults(fl.flat_grad, self.cfg.fault, self.rank, self.step_count,
                         self.group_active, self.cfg.seed + self.step_count,
                         cols=slice(b.offset, b.offset + b.length))
        st = self._opt_stream
        st.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(st):
            self._bucket_update(b)
        self._updated.add(b.index)

    def _bucket_update(self, b: Bucket) -> None:
        fl = self.flat
        m, s1, s2 = self._state(b.offset, b.length)
        K.agg_update(fl.flat_grad[:, b.offset:b.offset + b.length], combine="weighted", n=self.V,
                     opt=self._opt_args(gscale=1.0 / self.V), master=m, s1=s1, s2=s2,
                     param_out=fl.flat_param[b.offset:b.offset + b.length])

    def _flush_row(self) -> None:
        for b in self.flat.buckets:
            if b.index not in self._flushed:
                self._flush(b, complete=False)
        self._flushed.clear()

    def _launch_bucket(self, b: Bucket, inject: bool) -> None:
        fl = self.flat
        if inject and self.cfg.fault.kind != "none":
            apply_faults(fl.flat_grad, self.cfg.fault, self.rank, self.step_count,
                         self.group_active, self.cfg.seed + self.step_count,
                         cols=slice(b.offset, b.offset + b.length))
        if not self.group_active or self.topo == "gossip":
            self._pending[b.index] = None
            return
        g = fl.flat_grad[:, b.offset:b.offset + b.length]      # [V, L]
        if self.topo == "allreduce":
            src = g[0] if self.V == 1 else g.sum(0, dtype=torch.float32).to(g.dtype)
            if self.V > 1:
                g[0].copy_(src)
                src = g[0]
            self._pending[b.index] = dist.all_reduce(src, op=dist.ReduceOp.SUM, async_op=True)
        elif self.topo == "allgather":
            out = self.recv[b.index][: self.n]
            src = g if self.V > 1 else g[0]
            self._pending[b.index] = dist.all_gather_into_tensor(
                out.view(-1), src.contiguous().view(-1), async_op=True)
        else:  # sharded: chunk j of my bucket -> rank j; row (j*V+v) of recv = worker (j,v)'s shard r
            out = self.recv[b.index][: self.n]
            if self.V == 1:
                src = g[0]
            else:
                src = g.reshape(self.V, self.N, b.shard).transpose(0, 1).contiguous().view(-1)
            self._pending[b.index] = dist.all_to_all_single(out.view(-1), src, async_op=True)

    def _wait(self, b: Bucket) -> None:
        w = self._pending.get(b.index)
        if w is not None:
            w.wait()

    def _bucket_gram(self, b: Bucket) -> None:
        """Slot b of the per-bucket Gram partials, once its exchange has landed."""
        if b.index in self._gram_done:
            return
        self._wait(b)
        if self._fast_gram():
            # stage 1 only, into this bucket's own workspace, every argument resolved once
            # (persistent buffers: the host cost per bucket matters at small per-rank batches,
            # b256: ~700 launches / step); the stage-2 reduces of all buckets run as ONE launch
            # in _compute_weights
            X, length, ws = self._gram_args(b)
            self._gram_nblk[b.index] = lib().gram_partial(X, self.rows_total, length, ws,
                                                          self._pass_center())
        else:
            X = self._cclip_rows(b) if self.rule == "centered_clip" else self._rows(b)
            length = b.shard if self.topo == "sharded" else X.shape[1]
            K.gram(X, n=self.rows_total, D=length, out=self.Gb[b.index],
                   center=self._pass_center())
        self._gram_done.add(b.index)

    def _gram_args(self, b: Bucket):
        hit = self._gram_arg_cache.get(b.index)
        if hit is None:
            X = self._rows(b)
            length = b.shard if self.topo == "sharded" else X.shape[1]
            if X.data_ptr() % 16 or (X.stride(0) * X.element_size()) % 16 or X.stride(1) != 1:
                hit = False          # unaligned rows: K.gram pads a copy every call
            else:
                nbytes = int(lib().gram_workspace_bytes(self.rows_total, length))
                hit = (X, length, torch.empty(nbytes // 4 + 1, dtype=torch.float32,
                                              device=X.device))
            self._gram_arg_cache[b.index] = hit
        return hit or None

    def _fast_gram(self) -> bool:
        """GPU early Grams as per-bucket stage-1 launches + one deferred multi-bucket reduce."""
        if self._fast_gram_ok is None:
            self._fast_gram_ok = (self.device.type == "cuda" and self.rule != "centered_clip"
                                  and len(self.flat.buckets) <= 32
                                  and all(self._gram_args(b) is not None
                                          for b in self.flat.buckets))
        return self._fast_gram_ok

    def _poll_grams(self) -> None:
        """Gram partials of every bucket whose exchange has completed (non-blocking test), so
        they run during backward instead of after the last all-to-all."""
        for bi, w in list(self._pending.items()):
            if bi not in self._gram_done and w is not None and (self._gram_eager
                                                                or w.is_completed()):
                self._bucket_gram(self.flat.buckets[bi])
                self.early_grams += 1

    # ================================================================ optimizer args
    def _opt_args(self, gscale: float = 1.0) -> K.OptArgs:
        o = self.cfg.optim
        kind = o.name if o.name in ("sgd", "adam", "adamw") else "adamw"
        wd = o.weight_decay
        # 'adam' = torch.optim.Adam (L2 term in the gradient), 'adamw' = decoupled decay
        return K.OptArgs(kind=kind, lr=o.lr, momentum=o.momentum if kind == "sgd" else 0.0,
                         weight_decay=wd, nesterov=o.nesterov, first=self.step_count == 0,
                         beta1=o.betas[0], beta2=o.betas[1], eps=o.eps,
                         step=self.step_count + 1, gscale=gscale)

    def _state(self, off: int, length: int):
        m = self.master[off:off + length]
        s1 = self.s1[off:off + length] if self.s1 is not None else None
        s2 = self.s2[off:off + length] if self.s2 is not None else None
        return m, s1, s2

    # ================================================================ robust weights
    def _rows(self, b: Bucket) -> torch.Tensor:
        """Worker matrix of bucket b as seen by this rank ([rows_total, cols])."""
        fl = self.flat
        if self.topo == "sharded":
            if not self.group_active:
                # world 1: the local rows ARE the full workers; shard == bucket
                return fl.flat_grad[:, b.offset:b.offset + b.length]
            return self.recv[b.index]
        if self.topo == "allgather":
            if not self.group_active:
                return fl.flat_grad[:, b.offset:b.offset + b.length]
            return self.recv[b.index]
        raise RuntimeError("no worker matrix for this topology")

    def _cclip_rows(self, b: Bucket) -> torch.Tensor:
        """Worker rows plus the previous-aggregate row (centered clipping)."""
        X = self._rows(b)
        if X.shape[0] == self.rows_total:
            return X
        # world 1: stage the local rows into the recv-shaped buffer once
        if not self.recv:
            raise RuntimeError("centered_clip needs recv buffers")
        R = self.recv[b.index]
        R[: self.n].copy_(X)
        return R

    def _pass_center(self) -> Optional[torch.Tensor]:
        """Center row of this step's (first) Gram pass: the previous step's medoid (one centered
        pass per step), or None (uncentered) when no medoid is known yet or two passes are
        configured."""
        cfg = self.cfg.agg
        if cfg.centered_gram and self.have_center and not cfg.gram_two_pass:
            return self.center
        return None

    def _compute_weights(self, cols) -> None:
        """Gram over every bucket (accumulated in bucket order), all-reduced across shards,
        then weights."""
        cfg = self.cfg.agg
        center = self._pass_center()
        if self.early_gram:
            # per-bucket partials (computed during backward), summed in bucket order in one
            # launch: G = ((g0 + g1) + g2) ..., the same fp64 adds as accumulating bucket by bucket
            self._gram_queue.clear()
            for b, _, _ in cols:
                self._bucket_gram(b)
            if self._fast_gram():
                bs = self.flat.buckets
                lib().gram_reduce_multi([self._gram_args(b)[2] for b in bs],
                                        [self._gram_nblk[b.index] for b in bs], self.rows_total,
                                        self.G)
            else:
                K.gram_sum(self.Gb, self.G)
        else:
            self.G.zero_()
            for b, X, length in cols:
                K.gram(X, n=self.rows_total, D=length, out=self.G, accumulate=True, center=center)
        if self.group_active and self.topo == "sharded" and self.N > 1:
            dist.all_reduce(self.G)      # (one rank: the sum over ranks is G itself)
        if cfg.centered_gram and center is None:
            # no medoid yet (first step) or the two-pass scheme: a second pass relative to the
            # medoid of the uncentered G -- exact distances for near-duplicate workers (the rules
            # are translation invariant, so only the precision changes)
            K.gram_center(self.G, self.rows_total, out=self.center)
            self.G.zero_()
            for b, X, length in cols:
                K.gram(X, n=self.rows_total, D=length, out=self.G, accumulate=True,
                       center=self.center)
            if self.group_active and self.topo == "sharded" and self.N > 1:
                dist.all_reduce(self.G)
        rule = "bulyan_select" if self.rule == "bulyan" else self.rule
        m = cfg.m if cfg.m is not None else self.n - cfg.f
        iters = cfg.clip_iters if rule == "centered_clip" else cfg.iters
        # one launch: weights, selection counts and -- centered Gram -- the medoid of this step's
        # (precise) G, which centers the next step's single pass (computed on the device from the
        # all-reduced G, so every rank holds the same row). ``guard``: this G came from the single
        # pass centered on the PREVIOUS step's medoid, which a center turned Byzantine could
        # capture with huge finite values (weights.hip); a tripped guard zeroes this step's
        # weights and runs the next pass uncentered (center -1).
        K.robust_weights(self.G, rule, self.n, f=cfg.f, m=m, iters=iters, eps=cfg.eps,
                         tol=cfg.tol, tau=cfg.tau, w_out=self.w, scores=self.scores, sel=self.sel,
                         guard=center is not None,
                         center_out=self.center if cfg.centered_gram else None,
                         sel_counts=self.sel_counts)
        if cfg.centered_gram:
            self.have_center = True

    def _bucket_cols(self) -> list:
        out = []
        for b in self.flat.buckets:
            if self.rule == "centered_clip":
                X = self._cclip_rows(b)
            else:
                X = self._rows(b)
            length = b.shard if (self.topo == "sharded" and self.group_active) else X.shape[1]
            out.append((b, X, length))
        return out

    def _aggregate_update(self, b: Bucket, X: torch.Tensor, length: int, state_off: int,
                          param_out: torch.Tensor, opt: K.OptArgs,
                          gout: Optional[torch.Tensor]) -> None:
        cfg = self.cfg.agg
        m, s1, s2 = self._state(state_off, length)
        if self.rule in ("median", "trimmed_mean"):
            trim = cfg.trim if cfg.trim is not None else cfg.f
            lo, cnt = K.sorted_range(self.rule, self.n, trim)
            K.agg_update(X, combine="sorted", lo=lo, cnt=cnt, n=self.n, D=length, opt=opt,
                         master=m, s1=s1, s2=s2, param_out=param_out, gout=gout)
        elif self.rule == "bulyan":
            theta = self.n - 2 * cfg.f
            lo, cnt = K.sorted_range("trimmed_mean", theta, cfg.f)
            K.agg_update(X, combine="sorted", lo=lo, cnt=cnt, rows=self.sel[:theta], n=theta,
                         D=length, opt=opt, master=m, s1=s1, s2=s2, param_out=param_out,
                         gout=gout)
        else:  # mean and Gram-space rules: weighted
            K.agg_update(X, combine="weighted", w=self.w, n=self.rows_total, D=length, opt=opt,
                         master=m, s1=s1, s2=s2, param_out=param_out, gout=gout)

    def _aggregate_update_multi(self, segs, opt: K.OptArgs) -> None:
        """``_aggregate_update`` of several buckets in one launch: segs = (X, length, pout, soff)."""
        cfg = self.cfg.agg
        ks = [(X, length, soff, pout) for X, length, pout, soff in segs]
        st = dict(master=self.master, s1=self.s1, s2=self.s2, opt=opt)
        if self.rule in ("median", "trimmed_mean"):
            trim = cfg.trim if cfg.trim is not None else cfg.f
            lo, cnt = K.sorted_range(self.rule, self.n, trim)
            K.agg_update_multi(ks, combine="sorted", lo=lo, cnt=cnt, n=self.n, **st)
        elif self.rule == "bulyan":
            theta = self.n - 2 * cfg.f
            lo, cnt = K.sorted_range("trimmed_mean", theta, cfg.f)
            K.agg_update_multi(ks, combine="sorted", lo=lo, cnt=cnt, rows=self.sel[:theta],
                               n=theta, **st)
        else:
            K.agg_update_multi(ks, combine="weighted", w=self.w, n=self.rows_total, **st)

    # ================================================================ topologies
    def _step_allreduce(self) -> None:
        fl = self.flat
        for b in fl.buckets:
            self._wait(b)
        if not self.group_active and self.V > 1:
            fl.flat_grad[0].copy_(fl.flat_grad.float().sum(0).to(fl.dtype))
        opt = self._opt_args(gscale=1.0 / self.n)
        m, s1, s2 = self._state(0, fl.total)
        K.agg_update(fl.flat_grad[0], combine="weighted", n=1, opt=opt, master=m, s1=s1, s2=s2,
                     param_out=fl.flat_param)

    def _step_allgather(self) -> None:
        fl = self.flat
        for b in fl.buckets:
            self._wait(b)
        cols = self._bucket_cols()
        if self.rule in GRAM_RULES:
            self._compute_weights(cols)
        if self.record_stats:
            self._record_stats(cols)
        opt = self._opt_args()
        for b, X, length in cols:
            gout = self.gout[b.offset:b.offset + b.length] if self.gout is not None else None
            self._aggregate_update(b, X, length, b.offset, fl.flat_param[b.offset:b.offset + b.length],
                                   opt, gout)
            if self.rule == "centered_clip":
                X[self.n].copy_(gout.to(X.dtype))   # v0 <- new aggregate

    def _step_sharded(self) -> None:
        fl = self.flat
        for b in fl.buckets:
            self._wait(b)
        cols = self._bucket_cols()
        if self.rule in GRAM_RULES:
            self._compute_weights(cols)
        if self.record_stats:
            self._record_stats(cols)
        opt = self._opt_args()
        works = []
        order = list(reversed(cols)) if self.param_prefetch else cols

        def shard(b):
            if self.group_active:
                return fl.my_shard(fl.flat_param, b, self.rank), b.shard_offset
            return fl.flat_param[b.offset:b.offset + b.length], b.offset

        # every bucket's rule + optimizer step in ONE launch (centered clipping writes its
        # aggregate back into each bucket's rows, so it stays per bucket)
        fused = self.rule != "centered_clip" and 1 <= len(cols) <= 16 and self.device.type == "cuda"
        if fused:
            self._aggregate_update_multi([(X, length) + shard(b) for b, X, length in order], opt)
        # earliest layers (highest bucket index) first: the next forward needs them first
        for b, X, length in order:
            pout, soff = shard(b)
            if not fused:
                gout = self.gout[soff:soff + length] if self.gout is not None else None
                self._aggregate_update(b, X, length, soff, pout, opt, gout)
                if self.rule == "centered_clip":
                    X[self.n, :length].copy_(gout.to(X.dtype))
            if self.group_active and self.N > 1:
                # (one rank: the shard IS the bucket, the gather would copy it onto itself)
                full = fl.flat_param[b.offset:b.offset + b.length]
                work = dist.all_gather_into_tensor(full, pout, async_op=True)
                if self.param_prefetch:
                    self._ag_works[b.index] = work
                else:
                    works.append(work)
        for w in works:
            w.wait()

    def _setup_gossip(self) -> None:
        """Neighbour receive buffers. ring: left + right (full vectors); exp: ONE full vector
        (the step's single peer); exp_all: per-peer chunk buffers when synchronous (mixing runs
        chunk by chunk), full vectors in delayed mode (the exchange lands during the next step)."""
        fl, tc = self.flat, self.cfg.topology
        self.gossip_graph = tc.gossip_graph
        k = max_gossip_peers(self.gossip_graph, self.N)
        if k > K.GOSSIP_MAX_NBRS:
            raise ValueError(
                f"gossip graph {self.gossip_graph!r} at N={self.N} mixes {k} neighbours per step; "
                f"the mixing kernel takes at most {K.GOSSIP_MAX_NBRS} (use 'exp' or 'ring')")
        self._self_copy = self.N == 1 and dist.get_backend() != "nccl"
        # whole 128-byte lines per chunk: the mixing kernel reads 16-byte aligned vectors
        self._chunk = max(int(tc.gossip_chunk_mb * 1024 * 1024 // 2) // 64 * 64, 64)
        if self.gossip_graph == "ring":
            nbuf, full = 2, True
        elif self.gossip_graph == "exp":
            nbuf, full = 1, True
        else:
            nbuf = len(self._gossip_peers(0)[0])
            full = tc.gossip_async or tc.gossip_clip > 0
        size = fl.flat_param.numel() if full else min(self._chunk, fl.flat_param.numel())
        self.nb_bufs = [torch.empty(size, dtype=fl.flat_param.dtype, device=self.device)
                        for _ in range(nbuf)]
        self._nb_full = full

    def _gossip_peers(self, t: int):
        """(send-to, recv-from, mixing weights, self weight) of gossip step t; recv_from[k] is
        the rank whose parameters land in nb_bufs[k]."""
        return gossip_peers(self.gossip_graph, self.N, self.rank, t,
                            self.cfg.topology.gossip_weights)

    def _gossip_exchange(self, t: int, s: int, e: int, src: torch.Tensor, bufs, off: int):
        """Grouped send/recv of src[s:e] for step t; neighbour k's slice lands in
        bufs[k][s - off:e - off]."""
        send, recv, _, _ = self._gossip_peers(t)
        if self._self_copy:
            # 1-rank loopback group on gloo (no self pairs): the "received" slice is a copy;
            # RCCL sends to itself for real
            for k, q in enumerate(recv):
                if q == self.rank:
                    bufs[k][s - off:e - off].copy_(src[s:e])
            send = [q for q in send if q != self.rank]
            recv = [(k, q) for k, q in enumerate(recv) if q != self.rank]
        else:
            recv = list(enumerate(recv))
        ops = [dist.P2POp(dist.isend, src[s:e], q) for q in send]
        ops += [dist.P2POp(dist.irecv, bufs[k][s - off:e - off], q) for k, q in recv]
        return dist.batch_isend_irecv(ops) if ops else []

    def _gossip_mix(self, t: int, s: int, e: int, off: int = 0, send: bool = False) -> None:
        _, _, w, w0 = self._gossip_peers(t)
        K.gossip_mix_k(self.master[s:e], [b[s - off:e - off] for b in self.nb_bufs], w, w0,
                       self.cfg.topology.gossip_clip, param_out=self.flat.flat_param[s:e],
                       param_out2=self._send_buf[s:e] if send else None)

    def _step_gossip(self) -> None:
        fl = self.flat
        if not self.early_update:
            opt = self._opt_args(gscale=1.0 / self.V)
            m, s1, s2 = self._state(0, fl.total)
            K.agg_update(fl.flat_grad, combine="weighted", n=self.V, opt=opt, master=m, s1=s1,
                         s2=s2, param_out=fl.flat_param)
        if not self.group_active or not self._gossip_peers(self.step_count)[0]:
            return
        t = self.step_count
        clip = self.cfg.topology.gossip_clip
        chunk = self._chunk
        total = fl.total
        starts = list(range(0, total, chunk))

        def wait_all(reqs):
            for rq in reqs:
                for w in rq:
                    w.wait()

        if self.cfg.topology.gossip_async:
            # Delayed gossip: mix with the neighbour parameters that arrived during THIS step's
            # compute (sent at the end of the previous step, graph of step t - 1) and start the
            # next exchange, which overlaps the next forward/backward. The mix writes the new
            # parameters AND the send buffer in one pass (no snapshot copy of the parameters:
            # the next step's early updates overwrite them while the send is in flight). GPU: on
            # a side stream, bucket by bucket, earliest layers first; the next forward waits per
            # module (the prefetch hooks), so the mix overlaps it instead of preceding it.
            mixed = self._gossip_reqs is not None or self._gossip_restored
            ms = self._mix_stream
            if self._send_buf is None:
                self._send_buf = torch.empty_like(fl.flat_param)
            if ms is not None:
                ms.wait_stream(torch.cuda.current_stream(self.device))
            with (torch.cuda.stream(ms) if ms is not None else contextlib.nullcontext()):
                if mixed:
                    self._drain_gossip()        # (on the side stream: a device-side wait)
                    self._gossip_restored = False
                    if ms is None or clip > 0 or not self.param_prefetch:
                        # (clipping needs whole-vector neighbour distances)
                        self._gossip_mix(t - 1, 0, total, send=True)
                        if ms is not None and self.param_prefetch:
                            ev = _EventWork(ms)
                            for b in fl.buckets:
                                self._ag_works[b.index] = ev
                    else:
                        for b in reversed(fl.buckets):
                            self._gossip_mix(t - 1, b.offset, b.offset + b.length, send=True)
                            self._ag_works[b.index] = _EventWork(ms)
                else:
                    self._send_buf.copy_(fl.flat_param)   # first exchange: nothing mixed yet
                self._gossip_reqs = [self._gossip_exchange(t, s, min(s + chunk, total),
                                                           self._send_buf, self.nb_bufs, 0)
                                     for s in starts]
            if ms is not None and not self.param_prefetch:
                torch.cuda.current_stream(self.device).wait_stream(ms)
            return

        if clip > 0 and len(starts) > 1:
            # clipping needs whole-vector neighbour distances: exchange everything first
            wait_all([self._gossip_exchange(t, s, min(s + chunk, total), fl.flat_param,
                                            self.nb_bufs, 0) for s in starts])
            self._gossip_mix(t, 0, total)
            return
        if not self._nb_full:
            # per-peer chunk buffers: exchange chunk k, mix it, reuse the buffers for k + 1
            for s in starts:
                e = min(s + chunk, total)
                wait_all([self._gossip_exchange(t, s, e, fl.flat_param, self.nb_bufs, s)])
                self._gossip_mix(t, s, e, off=s)
            return
        reqs = self._gossip_exchange(t, starts[0], min(starts[0] + chunk, total), fl.flat_param,
                                     self.nb_bufs, 0)
        for k, s in enumerate(starts):
            e = min(s + chunk, total)
            nxt = (self._gossip_exchange(t, starts[k + 1], min(starts[k + 1] + chunk, total),
                                         fl.flat_param, self.nb_bufs, 0)
                   if k + 1 < len(starts) else None)
            for w in reqs:
                w.wait()
            self._gossip_mix(t, s, e)
            reqs = nxt

    # ================================================================ consensus table
    def _local_range(self, b: Bucket, length: int):
        """Flat-coordinate column range [lo, hi) of bucket b held in this rank's worker rows."""
        if self.topo == "sharded" and self.group_active:
            lo = b.offset + self.rank * b.shard
        else:
            lo = b.offset
        return lo, lo + length

    def _aggregate_only(self, b: Bucket, X: torch.Tensor, length: int) -> torch.Tensor:
        """The rule's aggregate of bucket b's local columns (fp32), without an update."""
        cfg = self.cfg.agg
        out = torch.empty(length, dtype=torch.float32, device=X.device)
        none = K.OptArgs(kind="none")
        if self.rule in ("median", "trimmed_mean"):
            trim = cfg.trim if cfg.trim is not None else cfg.f
            lo, cnt = K.sorted_range(self.rule, self.n, trim)
            K.agg_update(X, combine="sorted", lo=lo, cnt=cnt, n=self.n, D=length, opt=none,
                         gout=out)
        elif self.rule == "bulyan":
            theta = self.n - 2 * cfg.f
            lo, cnt = K.sorted_range("trimmed_mean", theta, cfg.f)
            K.agg_update(X, combine="sorted", lo=lo, cnt=cnt, rows=self.sel[:theta], n=theta,
                         D=length, opt=none, gout=out)
        else:
            K.agg_update(X, combine="weighted", w=self.w, n=self.rows_total, D=length, opt=none,
                         gout=out)
        return out

    def _record_stats(self, cols) -> None:
        """Per (parameter tensor, worker): squared gradient norm and squared distance to the
        aggregate, from the worker rows this rank holds; shard partial sums are all-reduced."""
        segs = self.flat.segments()
        n = self.n
        dev = self.device
        sq = torch.zeros(len(segs), n, dtype=torch.float64, device=dev)
        dd = torch.zeros(len(segs), n, dtype=torch.float64, device=dev)
        ag = torch.zeros(len(segs), dtype=torch.float64, device=dev)
        for b, X, length in cols:
            lo, hi = self._local_range(b, length)
            agg = self._aggregate_only(b, X, length)
            for k, (_, off, numel) in enumerate(segs):
                a, e = max(off, lo), min(off + numel, hi)
                if a >= e:
                    continue
                Xs = X[:n, a - lo:e - lo].double()
                gs = agg[a - lo:e - lo].double()
                sq[k] += (Xs * Xs).sum(1)
                dd[k] += ((Xs - gs[None]) ** 2).sum(1)
                ag[k] += (gs * gs).sum()
        if self.group_active and self.topo == "sharded":
            for t in (sq, dd, ag):
                dist.all_reduce(t)
        self.last_stats = {"names": [s[0] for s in segs], "sqnorm": sq.cpu(), "dist2": dd.cpu(),
                           "agg_sqnorm": ag.cpu(), "step": self.step_count,
                           "weights": self.w[:n].double().cpu(),
                           "scores": self.scores[:n].cpu() if self.rule in GRAM_RULES else None,
                           "sel_counts": self.sel_counts.cpu().clone()}
        self.record_stats = False

    def consensus_table(self):
        """The training-side analogue of the reference's standard output table
        (`composite_code/rnotebook/cml_targetaml_seanalysis.Rmd:627-633`, `:1297-1298`): one row
        per parameter tensor, one column per worker for its gradient norm and its distance to the
        robust aggregate, plus aggregate columns (aggregate norm, median worker norm, the worker
        farthest from the aggregate). Two trailing rows carry the per-worker Krum score and
        selection count / weight. Needs a step taken with ``record_stats = True``."""
        import pandas as pd
        st = self.last_stats
        if st is None:
            raise RuntimeError("no recorded step: set engine.record_stats = True before step()")
        n = self.n
        norm = st["sqnorm"].clamp_min(0).sqrt().numpy()
        d = st["dist2"].clamp_min(0).sqrt().numpy()
        df = pd.DataFrame(index=st["names"])
        for i in range(n):
            df[f"grad_norm_w{i}"] = norm[:, i]
        for i in range(n):
            df[f"dist_to_agg_w{i}"] = d[:, i]
        df["agg_norm"] = st["agg_sqnorm"].clamp_min(0).sqrt().numpy()
        df["median_worker_norm"] = np.median(norm, axis=1)
        df["farthest_worker"] = d.argmax(1)
        extra = pd.DataFrame(index=["(krum_score)", "(selection_count)", "(weight)"],
                             columns=df.columns, dtype=float)
        for i in range(n):
            if st["scores"] is not None:
                extra.loc["(krum_score)", f"grad_norm_w{i}"] = float(st["scores"][i])
            extra.loc["(selection_count)", f"grad_norm_w{i}"] = float(st["sel_counts"][i])
            extra.loc["(weight)", f"grad_norm_w{i}"] = float(st["weights"][i])
        out = pd.concat([df, extra])
        out.attrs["step"] = st["step"]
        return out

    def _drain_gossip(self) -> None:
        if self._gossip_reqs is not None:
            for rq in self._gossip_reqs:
                for w in rq:
                    w.wait()
            self._gossip_reqs = None

    # ================================================================ state
    def state_dict(self) -> dict:
        self.wait_params()
        sd = {"master": self.master, "step": self.step_count, "sel_counts": self.sel_counts,
              "rank": self.rank, "world": self.N, "topology": self.topo}
        if self.have_center:
            sd["gram_center"] = self.center
        if self.topo == "gossip" and self.cfg.topology.gossip_async and \
                (self._gossip_reqs is not None or self._gossip_restored):
            # delayed gossip: the exchange started at the end of the last step is part of the
            # state (the next step mixes with it); finish it and save what arrived
            self._drain_gossip()
            self._gossip_restored = True
            sd["gossip_nb"] = list(self.nb_bufs)
        if self.s1 is not None:
            sd["s1"] = self.s1
        if self.s2 is not None:
            sd["s2"] = self.s2
        if self.rule == "centered_clip":
            sd["v0"] = self.gout
        return sd

    def load_state_dict(self, sd: dict) -> None:
        if sd["world"] != self.N or sd["topology"] != self.topo:
            raise ValueError("checkpoint was written with a different world size / topology")
        self.master.copy_(sd["master"])
        if self.s1 is not None and "s1" in sd:
            self.s1.copy_(sd["s1"])
        if self.s2 is not None and "s2" in sd:
            self.s2.copy_(sd["s2"])
        self.step_count = int(sd["step"])
        self.sel_counts.copy_(sd["sel_counts"])
        if "gram_center" in sd:
            c = sd["gram_center"].reshape(-1)
            self.center[: c.numel()].copy_(c[:2])
            self.have_center = True
        if "v0" in sd and self.gout is not None:
            self.gout.copy_(sd["v0"])
        nb = sd.get("gossip_nb")
        if nb is None and "gossip_left" in sd:          # round-2 checkpoints (ring)
            nb = [sd["gossip_left"], sd["gossip_right"]]
        if nb is not None and self.topo == "gossip" and len(nb) == len(self.nb_bufs):
            self._drain_gossip()
            for dst, src in zip(self.nb_bufs, nb):
                dst.copy_(src)
            self._gossip_restored = True
        self.sync_params_from_master()

    def sync_params_from_master(self) -> None:
        """Rewrite the bf16 parameters from the fp32 master (after a checkpoint load)."""
        self.wait_params()
        fl = self.flat
        if self.topo == "sharded" and self.group_active:
            for b in fl.buckets:
                pout = fl.my_shard(fl.flat_param, b, self.rank)
                pout.copy_(self.master[b.shard_offset:b.shard_offset + b.shard].to(fl.dtype))
                dist.all_gather_into_tensor(fl.flat_param[b.offset:b.offset + b.length], pout)
        elif self.topo == "sharded":
            fl.flat_param.copy_(self.master.to(fl.dtype))
        else:
            fl.flat_param.copy_(self.master.to(fl.dtype))

    def close(self) -> None:
        self._drain_gossip()     # the in-flight delayed-gossip exchange
        self.wait_params()
        for h in self._prefetch_hooks:
            h.remove()
        self._prefetch_hooks = []
        for h in self._hooks:
            h.remove()
        self._hooks = []
