"""bench/configs.py under the headline harness's contract (CPU, gloo): ``--gpus N`` self-launch,
world-size exit, the mean all-reduce baseline with ``agg_overhead_vs_allreduce``, and the
cross-rank ``replicas_identical`` check, for every BASELINE.json config (tiny models of the same
families so the CPU runs stay short)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

TINY = {"mlp_median": ["--batch", "16"],
        "resnet_trimmed": ["--model", "resnet_tiny", "--batch", "4"],
        "resnet_mkrum": ["--model", "resnet_tiny", "--batch", "4"],
        "bert_geomed": ["--model", "bert_tiny", "--batch", "4", "--seq-len", "32"],
        "llama_gossip": ["--model", "llama_tiny", "--batch", "2", "--seq-len", "32",
                         "--bucket-mb", "8"]}


def _run(args, env=None, timeout=600):
    e = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, "bench/configs.py", *args], cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=timeout)


def _line(out):
    lines = [l for l in out.splitlines() if l.startswith("{") and '"config"' in l]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


CASES = [(c, 2) for c in sorted(TINY)] + [("mlp_median", 4), ("resnet_mkrum", 4)]


@pytest.mark.parametrize("config,n", CASES)
def test_config_contract(config, n):
    out = _run(["--config", config, "--gpus", str(n), "--steps", "2", "--warmup", "1",
                "--dist-backend", "gloo", *TINY[config]])
    assert out.returncode == 0, out.stderr[-3000:]
    r = _line(out.stdout)
    assert r["config"] == config and r["n_gpus"] == n and r["world_size_seen"] == n
    assert r["launcher"] == "self" and r["dist_backend"] == "gloo"
    assert r["allreduce_ms_per_step"] > 0 and r["agg_overhead_vs_allreduce"] is not None
    assert r["samples_per_s"] > 0 and r["steps"] == 2
    if config == "llama_gossip":
        assert r["replicas_identical"] is None and r["gossip_exchanged"]
    else:
        assert r["replicas_identical"] is True and r["allreduce_replicas_identical"] is True
        assert r["bucket_mb"] == 8
    if config == "resnet_mkrum" and n == 4:
        assert r["f"] == 1 and sum(r["selection_counts"]) > 0


def test_config_world_size_mismatch():
    out = _run(["--config", "mlp_median", "--gpus", "2", "--steps", "1", "--warmup", "0"],
               env={"WORLD_SIZE": "1", "RANK": "0"})
    assert out.returncode == 2 and "WORLD_SIZE" in out.stderr
