"""Weight gradients off the critical path of the backward (PerfPolicy.side_wgrad).

In a ResNet backward every layer produces a data gradient (the next layer's input: the critical
path) and a weight gradient that nothing later in the backward reads -- only the engine's
copy-on-ready capture. Launched on a second HIP stream, the weight-gradient kernels fill the CUs
that the data-gradient chain leaves idle (grid tails, small layer-3/4 grids at per-GPU batch 256)
instead of queueing behind it.

Safety, when ``run`` is used:
  * armed only by the consensus engine between ``zero_grad()`` and ``step()``: every parameter's
    ``.grad`` is None at the start of the backward and is read only by the engine's capture
    hooks, which ``join()`` (the compute stream waits for the side stream) before they copy, and
    at ``step()``; a callback queued on the autograd engine also joins at the end of every
    backward, so code reading ``.grad`` after ``backward()`` sees finished values;
  * every input tensor the side kernels read is ``record_stream``-ed on the side stream and the
    result on the compute stream, so the caching allocator reuses no memory still in use;
  * only for parameters used once per forward (ResNet conv weights): a second accumulation into
    the same ``.grad`` would read it on the compute stream before the join.
Each kernel is the same deterministic kernel on the same inputs: results are bit-identical.
"""
from __future__ import annotations

from typing import Callable, Dict, Optional

import torch

from ..perf import policy as _P

_STREAMS: Dict[torch.device, torch.cuda.Stream] = {}


class _State:
    armed: Optional[torch.device] = None
    used = False
    queued = False


_S = _State()


def arm(device: torch.device) -> None:
    """Engine: parameter gradients are None and captured by the engine's hooks from now on."""
    _S.armed = device if (device.type == "cuda" and _P().side_wgrad) else None


def disarm() -> None:
    join()
    _S.armed = None


def join() -> None:
    """The compute stream waits for every weight gradient launched on the side stream so far."""
    if not _S.used:
        return
    dev = _S.armed
    for d, s in _STREAMS.items():
        if dev is None or d == dev:
            torch.cuda.current_stream(d).wait_stream(s)
    _S.used = False


def _end_of_backward() -> None:
    _S.queued = False
    join()


def run(fn: Callable[[], torch.Tensor], *inputs: Optional[torch.Tensor]) -> torch.Tensor:
    """fn() (a weight gradient) on the side stream when armed, else inline."""
    dev = _S.armed
    x0 = next((t for t in inputs if t is not None), None)
    if dev is None or x0 is None or not x0.is_cuda or x0.device != dev:
        return fn()
    s = _STREAMS.get(dev)
    if s is None:
        s = _STREAMS[dev] = torch.cuda.Stream(device=dev)
    cur = torch.cuda.current_stream(dev)
    s.wait_stream(cur)
    with torch.cuda.stream(s):
        out = fn()
    for t in inputs:
        if t is not None and t.is_cuda:
            t.record_stream(s)
    out.record_stream(cur)
    _S.used = True
    if not _S.queued:
        _S.queued = True
        torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward)
    return out
