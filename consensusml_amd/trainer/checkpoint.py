"""Checkpoint / resume.

The reference persists stage results with R ``save()/load()`` of named result lists plus an
append-only standard table (`composite_code/rnotebook/cml_targetaml_seanalysis.Rmd:673`, `:778`,
`:1069`, `:1239`, `:1298`). Here a training checkpoint is a directory

    <root>/step_<k>/meta.json            config, world size, topology, step, wall time, the
                                         flat-buffer layout (buckets, shards, parameter offsets)
                                         and the PerfPolicy (kernel / fusion switches) in force
    <root>/step_<k>/rank<r>.pt           this rank's engine state (fp32 master / optimizer shard),
                                         model buffers (BN statistics), RNG states
    <root>/step_<k>/consensus_table.csv  per-parameter x per-worker gradient statistics of the
                                         checkpoint step (the standard table's training analogue)
    <root>/latest                        name of the newest complete checkpoint

written atomically: every rank writes into ``step_<k>.tmp``, a barrier, then rank 0 renames the
directory and rewrites ``latest``. Files are loaded with ``torch.load(weights_only=True)``.

Re-sharding: a checkpoint written at world N loads at any world M. The saved layout tells where
every parameter's values sit in each rank's shard vector; the loader rebuilds full per-parameter
fp32 state (master, momentum / Adam moments, centered-clipping v0) from the N files and cuts the
current rank's shard (sharded topology) or the full vector (replicated topologies) out of it in
the CURRENT layout (bucket padding depends on the world size, so layouts differ between worlds).
Gossip replicas are per-rank by design: rank r takes the state of saved rank r mod N.
"""
from __future__ import annotations

import json
import os
import shutil
import time
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..parallel.dist import barrier
from ..perf import policy

STATE_KEYS = ("master", "s1", "s2", "v0")


def _rng_state(device: torch.device) -> dict:
    st = {"cpu": torch.get_rng_state()}
    if device.type == "cuda":
        st["cuda"] = torch.cuda.get_rng_state(device)
    return st


def layout_of(engine) -> dict:
    fl = engine.flat
    return {"world": engine.N, "topology": engine.topo,
            "total": fl.total, "shard_total": fl.shard_total,
            "buckets": [[b.offset, b.length, b.shard, b.shard_offset] for b in fl.buckets],
            "params": [[n, o, k] for n, o, k in fl.segments()]}


def save_checkpoint(root: str, engine, cfg, extra: Optional[dict] = None,
                    gens: Optional[list] = None, table=None) -> str:
    rank = engine.rank
    step = engine.step_count
    final = os.path.join(root, f"step_{step}")
    tmp = final + ".tmp"
    if rank == 0:
        os.makedirs(root, exist_ok=True)
        if os.path.exists(tmp):
            shutil.rmtree(tmp)
        os.makedirs(tmp)
    barrier()
    os.makedirs(tmp, exist_ok=True)
    buffers = {k: v.detach().cpu() for k, v in engine.model.named_buffers()}
    state = {
        "engine": {k: (v.detach().cpu() if torch.is_tensor(v) else v)
                   for k, v in engine.state_dict().items()},
        "buffers": buffers,
        "rng": _rng_state(engine.device),
        "gens": [g.get_state() for g in gens] if gens else None,
        "extra": extra or {},
    }
    path = os.path.join(tmp, f"rank{rank}.pt")
    torch.save(state, path + ".part")
    os.replace(path + ".part", path)
    if rank == 0:
        meta = {"step": step, "world": engine.N, "topology": engine.topo, "rule": engine.rule,
                "time": time.time(), "config": json.loads(cfg.to_json()),
                "params": engine.flat.real_numel, "layout": layout_of(engine),
                "perf_policy": policy().to_dict()}
        with open(os.path.join(tmp, "meta.json"), "w") as fh:
            json.dump(meta, fh, indent=1)
        if table is not None:
            table.to_csv(os.path.join(tmp, "consensus_table.csv"))
    barrier()
    if rank == 0:
        if os.path.exists(final):
            shutil.rmtree(final)
        os.replace(tmp, final)
        with open(os.path.join(root, "latest.part"), "w") as fh:
            fh.write(os.path.basename(final))
        os.replace(os.path.join(root, "latest.part"), os.path.join(root, "latest"))
    barrier()
    return final


def latest_checkpoint(root: str) -> Optional[str]:
    p = os.path.join(root, "latest")
    if not os.path.exists(p):
        return None
    with open(p) as fh:
        name = fh.read().strip()
    d = os.path.join(root, name)
    return d if os.path.isdir(d) else None


def _load_rank(path: str, r: int) -> dict:
    return torch.load(os.path.join(path, f"rank{r}.pt"), map_location="cpu", weights_only=True)


def _full_flat(vec_by_rank: List[torch.Tensor], lay: dict) -> torch.Tensor:
    """Full flat vector (saved layout) from per-rank shard vectors (sharded topology)."""
    out = torch.zeros(lay["total"], dtype=vec_by_rank[0].dtype)
    for off, length, shard, soff in lay["buckets"]:
        for r, v in enumerate(vec_by_rank):
            out[off + r * shard: off + (r + 1) * shard] = v[soff:soff + shard]
    return out


def _relayout(src_full: torch.Tensor, src_lay: dict, engine) -> torch.Tensor:
    """Move per-parameter values from the saved flat layout into the engine's flat layout, then
    cut this rank's shard vector (sharded) or keep the full vector."""
    fl = engine.flat
    dst = torch.zeros(fl.total, dtype=src_full.dtype)
    src = {n: (o, k) for n, o, k in src_lay["params"]}
    for n, o, k in fl.segments():
        if n not in src:
            raise ValueError(f"checkpoint has no parameter {n!r}")
        so, sk = src[n]
        if sk != k:
            raise ValueError(f"parameter {n!r} has {sk} elements in the checkpoint, {k} now")
        dst[o:o + k] = src_full[so:so + k]
    if engine.topo == "sharded" and engine.group_active:
        return fl.gather_shard_vector(dst, engine.rank)
    return dst


def _resharded_state(path: str, meta: dict, engine) -> Dict[str, object]:
    lay = meta.get("layout")
    if lay is None:
        raise ValueError("checkpoint predates layout metadata: it can only be loaded at world "
                         f"{meta['world']}")
    N = lay["world"]
    src_sharded = lay["topology"] == "sharded" and N > 1
    if lay["topology"] == "gossip":
        ranks = [engine.rank % N]
    elif src_sharded:
        ranks = list(range(N))
    else:
        ranks = [0]                       # replicated state: any rank's copy
    states = {r: _load_rank(path, r) for r in ranks}
    first = states[ranks[0]]
    es: Dict[str, object] = {}
    for key in STATE_KEYS:
        if key not in first["engine"]:
            continue
        if src_sharded:
            full = _full_flat([states[r]["engine"][key] for r in ranks], lay)
        else:
            full = first["engine"][key]
        es[key] = _relayout(full, lay, engine)
    es["step"] = int(first["engine"]["step"])
    sc = first["engine"]["sel_counts"]
    n = engine.sel_counts.numel()
    sel = torch.zeros(n, dtype=sc.dtype)
    sel[:min(n, sc.numel())] = sc[:min(n, sc.numel())]
    es["sel_counts"] = sel
    se = first["engine"]
    nb = se.get("gossip_nb") or ([se["gossip_left"], se["gossip_right"]]
                                  if "gossip_left" in se else None)
    if lay["topology"] == "gossip" and engine.topo == "gossip" and nb is not None:
        # delayed gossip: the neighbour parameters that arrived before the save (saved rank
        # r mod N's). At another world size the neighbours are other ranks, so the first mix
        # after the load uses these as the nearest available neighbour snapshot (the engine
        # takes them when the graph keeps the same number of receive buffers).
        es["gossip_nb"] = [_relayout(v, lay, engine) for v in nb]
    es["world"] = engine.N
    es["topology"] = engine.topo
    mine = states.get(engine.rank % N, first)
    return {"engine": es, "buffers": mine["buffers"], "rng": mine["rng"],
            "gens": mine.get("gens"), "extra": mine.get("extra", {})}


def load_checkpoint(path: str, engine, gens: Optional[list] = None) -> dict:
    """Load ``path`` (a step directory or a root with ``latest``) into the engine. A checkpoint of
    another world size (or topology) is re-sharded on load."""
    if os.path.exists(os.path.join(path, "latest")):
        path = latest_checkpoint(path)
    with open(os.path.join(path, "meta.json")) as fh:
        meta = json.load(fh)
    same = meta["world"] == engine.N and meta["topology"] == engine.topo
    if same:
        st = _load_rank(path, engine.rank)
    else:
        st = _resharded_state(path, meta, engine)
    es = {k: (v.to(engine.device) if torch.is_tensor(v) else v) for k, v in st["engine"].items()}
    engine.load_state_dict(es)
    bufs = dict(engine.model.named_buffers())
    for k, v in st["buffers"].items():
        if k in bufs:
            bufs[k].copy_(v.to(bufs[k].device))
    torch.set_rng_state(st["rng"]["cpu"])
    if "cuda" in st["rng"] and engine.device.type == "cuda":
        torch.cuda.set_rng_state(st["rng"]["cuda"], engine.device)
    if same and gens and st.get("gens"):
        for g, s in zip(gens, st["gens"]):
            g.set_state(s)
    return {"meta": meta, "extra": st.get("extra", {}), "resharded": not same}
