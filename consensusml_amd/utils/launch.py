"""One-process-per-GPU self-launch shared by the benchmark harnesses (bench.py,
bench/configs.py): ``--gpus N`` without an external launcher starts N ranks of the calling
script with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* on 127.0.0.1.

The parent never touches the GPU (nothing here initialises HIP: the children are started with
``subprocess``, never ``exec``), waits for every rank and returns the first non-zero exit code;
once one rank has failed the others get ``CML_BENCH_KILL_GRACE_S`` (60 s) to fail on their own
(a collective timeout) and are then killed, so a broken rank can never leave the run hanging.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional


def self_launch(n: int, script: str, argv: Optional[List[str]] = None, tag: str = "bench") -> int:
    argv = sys.argv[1:] if argv is None else argv
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0",
                   CML_BENCH_SELF_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(script), *argv],
                                      env=env, start_new_session=True))
    print(f"[{tag}] self-launched {n} ranks (pids {[p.pid for p in procs]}, port {port})",
          file=sys.stderr, flush=True)
    rc, failed_at = 0, None
    grace = float(os.environ.get("CML_BENCH_KILL_GRACE_S", "60"))
    alive = set(range(n))
    try:
        while alive:
            for r in sorted(alive):
                c = procs[r].poll()
                if c is None:
                    continue
                alive.discard(r)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    failed_at = time.monotonic()
                    print(f"[{tag}] rank {r} exited with {c}", file=sys.stderr, flush=True)
            if alive and failed_at is not None and time.monotonic() - failed_at > grace:
                for r in alive:
                    print(f"[{tag}] killing rank {r} (pid {procs[r].pid})", file=sys.stderr,
                          flush=True)
                    os.killpg(procs[r].pid, signal.SIGKILL)
                for r in alive:
                    procs[r].wait()
                alive.clear()
            time.sleep(0.2)
    except KeyboardInterrupt:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
        raise
    return rc


def launch_or_check(gpus: int, script: str, tag: str = "bench") -> int:
    """Resolve the rank layout of a harness started with ``--gpus N``: no WORLD_SIZE and N > 1
    -> self-launch N ranks and exit with their code; WORLD_SIZE != N -> exit 2. Returns the
    world size otherwise."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and gpus > 1:
        sys.exit(self_launch(gpus, script, tag=tag))
    world = int(world_env or "1")
    if world != gpus:
        print(f"[{tag}] error: --gpus {gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    return world


def param_checksum(flat_param):
    """Exact position-weighted int64 checksum of a bf16 / fp16 parameter vector's bits (equal iff
    bit-identical, up to a negligible collision chance)."""
    import torch
    bits = flat_param.view(torch.int16).to(torch.int64)
    idx = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) % 65521 + 1
    return torch.stack([(bits * idx).sum(), bits.sum()])


def replicas_identical(flat_param) -> bool:
    """Every rank holds bit-identical parameters (collective: call on every rank)."""
    import torch
    import torch.distributed as dist
    cs = param_checksum(flat_param)
    hi, lo = cs.clone(), cs.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    return bool(torch.equal(hi, lo))
