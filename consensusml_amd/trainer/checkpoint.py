"""Checkpoint / resume.

The reference persists stage results with R ``save()/load()`` of named result lists plus an
append-only standard table (`composite_code/rnotebook/cml_targetaml_seanalysis.Rmd:673`, `:778`,
`:1069`, `:1239`, `:1298`). Here a training checkpoint is a directory

    <root>/step_<k>/meta.json        config, world size, topology, step, wall time (rank 0)
    <root>/step_<k>/rank<r>.pt       this rank's engine state (fp32 master / optimizer shard),
                                     model buffers (BN statistics), RNG states
    <root>/latest                    name of the newest complete checkpoint

written atomically: every rank writes into ``step_<k>.tmp``, a barrier, then rank 0 renames the
directory and rewrites ``latest``. Files are loaded with ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import json
import os
import shutil
import time
from typing import Optional

import torch
import torch.distributed as dist

from ..parallel.dist import barrier


def _rng_state(device: torch.device) -> dict:
    st = {"cpu": torch.get_rng_state()}
    if device.type == "cuda":
        st["cuda"] = torch.cuda.get_rng_state(device)
    return st


def save_checkpoint(root: str, engine, cfg, extra: Optional[dict] = None,
                    gens: Optional[list] = None) -> str:
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
                "params": engine.flat.real_numel}
        with open(os.path.join(tmp, "meta.json"), "w") as fh:
            json.dump(meta, fh, indent=1)
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


def load_checkpoint(path: str, engine, gens: Optional[list] = None) -> dict:
    """Load ``path`` (a step directory or a root with ``latest``) into the engine."""
    if os.path.exists(os.path.join(path, "latest")):
        path = latest_checkpoint(path)
    with open(os.path.join(path, "meta.json")) as fh:
        meta = json.load(fh)
    if meta["world"] != engine.N:
        raise ValueError(f"checkpoint world {meta['world']} != current world {engine.N}")
    st = torch.load(os.path.join(path, f"rank{engine.rank}.pt"), map_location="cpu",
                    weights_only=True)
    es = {k: (v.to(engine.device) if torch.is_tensor(v) else v) for k, v in st["engine"].items()}
    engine.load_state_dict(es)
    bufs = dict(engine.model.named_buffers())
    for k, v in st["buffers"].items():
        if k in bufs:
            bufs[k].copy_(v.to(bufs[k].device))
    torch.set_rng_state(st["rng"]["cpu"])
    if "cuda" in st["rng"] and engine.device.type == "cuda":
        torch.cuda.set_rng_state(st["rng"]["cuda"], engine.device)
    if gens and st.get("gens"):
        for g, s in zip(gens, st["gens"]):
            g.set_state(s)
    return {"meta": meta, "extra": st.get("extra", {})}
