"""Structured JSONL step logs and per-phase GPU timers.

The reference only prints (`scripts/model_comp.py:30-33`, sklearn ``verbose=1`` timings at
`scripts/model_walkthrough.ipynb:195`). Here every step can emit one JSON object (throughput,
phase breakdown from HIP events, aggregation overhead, selection statistics).
"""
from __future__ import annotations

import json
import os
import time
from contextlib import contextmanager
from typing import Dict, List, Optional

import torch


class JsonlLogger:
    def __init__(self, path: Optional[str], rank: int = 0, all_ranks: bool = False):
        self.path = path
        self.enabled = path is not None and (rank == 0 or all_ranks)
        self.rank = rank
        if self.enabled:
            d = os.path.dirname(path)
            if d:
                os.makedirs(d, exist_ok=True)
            self._fh = open(path, "a", buffering=1)

    def log(self, **kw) -> None:
        if not self.enabled:
            return
        kw.setdefault("time", time.time())
        kw.setdefault("rank", self.rank)
        self._fh.write(json.dumps(kw, default=_default) + "\n")

    def close(self) -> None:
        if self.enabled:
            self._fh.close()
            self.enabled = False


def _default(o):
    if torch.is_tensor(o):
        return o.tolist()
    return str(o)


class PhaseTimer:
    """Records HIP events around named phases; ``summary()`` syncs once and returns ms per phase."""

    def __init__(self, device: torch.device, enabled: bool = True):
        self.cuda = device.type == "cuda"
        self.enabled = enabled
        self._events: List[tuple] = []
        self._cpu: Dict[str, float] = {}

    @contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        if self.cuda:
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            yield
            b.record()
            self._events.append((name, a, b))
        else:
            t = time.perf_counter()
            yield
            self._cpu[name] = self._cpu.get(name, 0.0) + (time.perf_counter() - t) * 1e3

    def summary(self, reset: bool = True) -> Dict[str, float]:
        out = dict(self._cpu)
        if self._events:
            torch.cuda.synchronize()
            for name, a, b in self._events:
                out[name] = out.get(name, 0.0) + a.elapsed_time(b)
        if reset:
            self._events.clear()
            self._cpu.clear()
        return out
