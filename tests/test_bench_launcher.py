"""bench.py's own launcher (CPU, gloo): ``--gpus N`` without WORLD_SIZE starts N ranks itself and
the run can never silently measure fewer ranks than asked for; a failing rank ends the whole run
with a non-zero exit instead of a hang. Plus the gossip-graph peer limits."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = ["--dist-backend", "gloo", "--model", "mlp", "--batch", "8", "--steps", "2",
        "--warmup", "1", "--no-miopen-find", "--b256-batch", "0"]


def _bench(args, env=None, timeout=300):
    e = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=timeout)


def _line(out):
    lines = [l for l in out.splitlines() if l.startswith("{") and '"metric"' in l]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 4])
def test_self_launch_world_size(n):
    out = _bench(["--gpus", str(n), *TINY])
    assert out.returncode == 0, out.stderr[-3000:]
    r = _line(out.stdout)
    assert r["n_gpus"] == n and r["world_size_seen"] == n and r["launcher"] == "self"
    assert r["replicas_identical"] is True and r["dist_backend"] == "gloo"
    assert r["config"]["parallelism"] == f"dp{n}" and r["config"]["global_batch"] == 8 * n
    if n >= 4:   # Krum with a real Byzantine budget
        assert r["config"]["f"] == 1 and r["selection"]["selected_last_step"] >= 1


def test_world_size_mismatch_fails():
    out = _bench(["--gpus", "2", *TINY], env={"WORLD_SIZE": "1", "RANK": "0"})
    assert out.returncode == 2 and "WORLD_SIZE" in out.stderr


def test_failed_rank_ends_run():
    """Rank 1 dies right after the process group exists; rank 0 must not hang in its next
    collective: the run ends non-zero (rank 1's code) well before the collective timeout."""
    out = _bench(["--gpus", "2", *TINY, "--timeout", "120"],
                 env={"CML_BENCH_FAIL_RANK": "1", "CML_BENCH_KILL_GRACE_S": "5"}, timeout=100)
    assert out.returncode == 7, out.stderr[-2000:]
    assert not any(l.startswith("{") for l in out.stdout.splitlines())


def test_gossip_peer_limits():
    from consensusml_amd.ops.kernels import GOSSIP_MAX_NBRS
    from consensusml_amd.parallel.engine import gossip_peers, max_gossip_peers
    assert max_gossip_peers("exp_all", 8) == 5
    assert max_gossip_peers("exp_all", 16) == 7
    assert max_gossip_peers("exp_all", 32) == 9 > GOSSIP_MAX_NBRS
    assert max_gossip_peers("exp", 32) == 1 and max_gossip_peers("ring", 64) == 2
    for N in (2, 3, 5, 8, 13, 32):
        for t in range(6):
            send = [gossip_peers("exp", N, r, t)[0][0] for r in range(N)]
            recv = [gossip_peers("exp", N, r, t)[1][0] for r in range(N)]
            for r in range(N):   # every send has its matching receive
                assert recv[send[r]] == r


def test_exp_all_rejected_above_kernel_limit():
    """exp_all at N = 32 needs 9 neighbour buffers: refused when the engine is built, before any
    buffer or collective (the mixing kernel reads at most 8)."""
    from consensusml_amd import TrainConfig
    from consensusml_amd.parallel.engine import ConsensusEngine
    cfg = TrainConfig()
    cfg.topology.kind = "gossip"
    cfg.topology.gossip_graph = "exp_all"
    eng = ConsensusEngine.__new__(ConsensusEngine)
    eng.cfg, eng.N, eng.rank = cfg, 32, 0
    eng.flat = None
    with pytest.raises(ValueError, match="at most 8"):
        ConsensusEngine._setup_gossip(eng)
