"""Process-group bootstrap: one process per GPU, torch.distributed over RCCL (backend "nccl" on
ROCm) or gloo for the CPU plumbing config.

The launcher is ``torchrun`` (or ``python -m torch.distributed.run``) with
``--master-addr 127.0.0.1``; RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* come from the environment.
``HSA_ENABLE_IPC_MODE_LEGACY=0`` must stay exported for RCCL on this platform.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"
    # a 1-rank process group that the engine drives exactly like a multi-rank one (every
    # all-to-all / all-gather / all-reduce / send-recv is issued, to this rank itself): the RCCL
    # code path of the N > 1 engine, runnable on a single GPU
    loopback: bool = False

    @property
    def is_master(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return (self.world > 1 or self.loopback) and dist.is_available() and \
            dist.is_initialized()


_INFO: Optional[DistInfo] = None


def init_distributed(backend: str = "auto", device: Optional[str] = None,
                     timeout_s: float = 1800.0, loopback: bool = False) -> DistInfo:
    """Initialise (once) and return this process's DistInfo.

    ``loopback``: with WORLD_SIZE 1, still create a (1-rank, in-process store) process group so
    the engine issues its collectives -- over RCCL when the backend is nccl -- to itself.
    ``timeout_s`` bounds every collective: a rank that stops answering ends the run with an
    error (RCCL: the watchdog aborts the communicator and the process) instead of a hang."""
    global _INFO
    if _INFO is not None:
        return _INFO
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if device is None:
        use_gpu = backend != "gloo" and torch.cuda.is_available()
        dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1)) if use_gpu \
            else torch.device("cpu")
    else:
        dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    if backend == "auto":
        backend = "nccl" if dev.type == "cuda" else "gloo"
    if backend == "nccl" and dev.type == "cuda" and local >= torch.cuda.device_count():
        raise RuntimeError(f"nccl (RCCL) needs one GPU per rank: local rank {local} of "
                           f"{world} but {torch.cuda.device_count()} visible GPU(s)")
    loop = bool(loopback and world == 1)
    if (world > 1 or loop) and not dist.is_initialized():
        # surface collective failures as errors (the default already does on recent torch)
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        kw = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if loop:
            kw["store"] = dist.HashStore()
        else:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29500")
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    active = world > 1 or loop
    _INFO = DistInfo(rank, world, local, dev, backend if active else "none", loopback=loop)
    return _INFO


def get_info() -> DistInfo:
    return _INFO if _INFO is not None else DistInfo()


def set_info(info: DistInfo) -> None:
    """Install a DistInfo (tests that create process groups themselves)."""
    global _INFO
    _INFO = info


def barrier() -> None:
    if dist.is_available() and dist.is_initialized():
        if get_info().device.type == "cuda" and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[get_info().device.index])
        else:
            dist.barrier()


def all_reduce_max(x: float) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=get_info().device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def monitored_barrier(timeout_s: float = 60.0) -> None:
    """Hang detector: on gloo, names the ranks that failed to arrive."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    if dist.get_backend() == "gloo":
        dist.monitored_barrier(timeout=datetime.timedelta(seconds=timeout_s), wait_all_ranks=True)
    else:
        barrier()


def shutdown() -> None:
    global _INFO
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _INFO = None
