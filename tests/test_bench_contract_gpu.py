"""bench.py's driver contract (one JSON line on rank 0 with the required keys), at a tiny shape:
1 rank with the virtual-worker Krum block, and 2 ranks sharing cuda:0 over gloo (the N > 1 fields:
dist_backend, world_size_seen, replicas_identical, engine_step_ms)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric": str, "value": float, "unit": str, "n_gpus": int, "steps": int, "warmup": int,
        "ms_per_step": float, "higher_is_better": bool, "scaling": str, "dtype": str,
        "data": str, "config": dict}
SMALL = ["--batch", "16", "--image-size", "64", "--steps", "2", "--warmup", "1",
         "--no-miopen-find", "--b256-batch", "8", "--b256-steps", "2"]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_line(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{") and '"metric"' in l]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def _check(r: dict, n: int):
    for k, t in KEYS.items():
        assert k in r and isinstance(r[k], t), (k, r.get(k))
    assert "vs_baseline" in r
    assert r["n_gpus"] == n and r["steps"] == 2 and r["warmup"] == 1
    assert r["value"] > 0 and r["ms_per_step"] > 0 and r["higher_is_better"] is True
    for k in ("model", "global_batch", "seq_len", "parallelism"):
        assert k in r["config"]
    assert r["config"]["global_batch"] == 16 * n
    # the communication-visible small-batch block (here batch 8 per rank)
    for k in ("b256_samples_per_s", "b256_ms_per_step", "b256_allreduce_ms_per_step",
              "b256_agg_overhead_vs_allreduce", "b256_engine_step_ms"):
        assert isinstance(r[k], float), (k, r.get(k))
    assert r["b256_config"]["global_batch"] == 8 * n and r["b256_loss_finite"] is True


def test_bench_single_rank_contract(cuda):
    env = dict(os.environ, PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, "bench.py", *SMALL, "--virtual-batch", "8",
                          "--virtual-steps", "2"], cwd=ROOT, env=env, capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    r = _json_line(out.stdout)
    _check(r, 1)
    assert r["krum_n8_virtual_config"]["workers"] == 8 and r["krum_n8_virtual_config"]["f"] == 2
    assert r["krum_n8_virtual_loss_finite"] is True


def test_bench_two_ranks_gloo_contract(cuda):
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--dist-backend", "gloo", *SMALL]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    r = _json_line(out.stdout)
    _check(r, 2)
    assert r["dist_backend"] == "gloo" and r["world_size_seen"] == 2
    assert r["replicas_identical"] is True and r["engine_step_ms"] >= 0
    assert r["b256_replicas_identical"] is True
