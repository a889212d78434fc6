"""Multi-process tests on gloo, world_size 2, 3, 4 and 8 (BASELINE config 1: 2-layer MLP, coordinate-wise
median) — the "multi-node without a cluster" fixture of SURVEY.md §4.4 item 3.

A run with R ranks x 1 worker must produce bit-for-bit (fp32) the same parameters as 1 rank x R
virtual workers fed the same per-worker data: that pins the all-to-all / all-gather / all-reduce
plumbing, the shard layout and the Gram all-reduce to the single-process semantics.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from consensusml_amd import TrainConfig


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(rule, topo, V, f, steps, fault="none", byz=()):
    cfg = TrainConfig()
    cfg.dtype = "fp32"
    cfg.virtual_workers = V
    cfg.agg.rule = rule
    cfg.agg.f = f
    cfg.topology.kind = "gossip" if topo == "gossip_async" else topo
    cfg.topology.gossip_async = topo == "gossip_async"
    cfg.topology.bucket_mb = 0.002      # several buckets even for the tiny MLP
    cfg.optim.lr = 0.1
    cfg.batch_per_worker = 16
    cfg.model.extra = {"classes": 2}
    cfg.fault.kind = fault
    cfg.fault.ranks = list(byz)
    cfg.backend = "gloo"
    cfg.steps = steps
    return cfg


def _worker(rank, world, port, rule, topo, f, steps, out_dir, fault, byz, ckpt, prefetch=True,
            early_gram=True):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from consensusml_amd.parallel import dist as D
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    D._INFO = None
    info = D.init_distributed("gloo")
    cfg = _cfg(rule, topo, 1, f, steps, fault, byz)
    cfg.topology.param_prefetch = prefetch
    cfg.topology.early_gram = early_gram
    if ckpt:
        cfg.ckpt_dir = os.path.join(out_dir, "ckpt")
    tr = ConsensusTrainer(cfg, info=info)
    # early_gram: compute every bucket's Gram in its hook (the timing-dependent path, forced)
    tr.engine._gram_eager = early_gram
    if ckpt:
        tr.fit(steps // 2, log_every=0)
        tr.save()
        tr2 = ConsensusTrainer(cfg, info=info)
        tr2.load(cfg.ckpt_dir)
        tr2.fit(steps, log_every=0)
        tr = tr2
    else:
        tr.fit(steps, log_every=0)
    params = [p.detach().clone() for p in tr.model.parameters()]
    torch.save({"params": params, "sel": tr.engine.sel_counts.clone(),
                "early_grams": tr.engine.early_grams},
               os.path.join(out_dir, f"r{rank}.pt"))
    D.monitored_barrier(30)
    dist.destroy_process_group()


def _run_world(world, rule, topo, f, steps, tmp, fault="none", byz=(), ckpt=False,
               prefetch=True, early_gram=True):
    port = _free_port()
    mp.spawn(_worker, args=(world, port, rule, topo, f, steps, str(tmp), fault, list(byz), ckpt,
                            prefetch, early_gram), nprocs=world, join=True)
    return [torch.load(os.path.join(tmp, f"r{r}.pt"), weights_only=True) for r in range(world)]


def _single(world, rule, topo, f, steps, fault="none", byz=()):
    from consensusml_amd.parallel.dist import DistInfo
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    cfg = _cfg(rule, topo, world, f, steps, fault, byz)
    tr = ConsensusTrainer(cfg, info=DistInfo(0, 1, 0, torch.device("cpu"), "none"))
    tr.fit(steps, log_every=0)
    return [p.detach().clone() for p in tr.model.parameters()]


@pytest.mark.parametrize("topo,rule,world,f", [
    ("sharded", "median", 2, 0),          # BASELINE config 1
    ("allgather", "median", 2, 0),
    ("allreduce", "mean", 2, 0),
    ("sharded", "krum", 3, 0),
    ("sharded", "geomed", 3, 0),
    ("allgather", "multi_krum", 3, 1),
    ("sharded", "trimmed_mean", 3, 1),
    ("sharded", "multi_krum", 4, 1),
    ("sharded", "krum", 8, 1),            # the bench's topology / rule at the node's 8 ranks
])
def test_distributed_equals_virtual(tmp_path, topo, rule, world, f):
    res = _run_world(world, rule, topo, f, 6, tmp_path)
    single = _single(world, rule, topo, f, 6)
    for r in range(world):
        for a, b in zip(res[r]["params"], single):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_byzantine_rank_excluded_gloo(tmp_path):
    res = _run_world(3, "krum", "sharded", 0, 8, tmp_path, fault="sign_flip", byz=[1])
    assert res[0]["sel"][1].item() == 0
    for a, b in zip(res[0]["params"], res[2]["params"]):
        torch.testing.assert_close(a, b)


@pytest.mark.parametrize("topo", ["gossip", "gossip_async"])
def test_gossip_ring_runs(tmp_path, topo):
    res = _run_world(3, "mean", topo, 0, 6, tmp_path)
    for r in range(3):
        assert all(torch.isfinite(p).all() for p in res[r]["params"])
    # gossip pulls the replicas together: spread across ranks stays small vs the weights
    for ps in zip(*[res[r]["params"] for r in range(3)]):
        spread = torch.stack(ps).std(0).max()
        assert spread < 0.1 * max(p.abs().max() for p in ps) + 1e-3


def test_checkpoint_resume_gloo(tmp_path):
    """save at step 3, reload into a fresh trainer, continue to 6 == uninterrupted 6 steps."""
    res = _run_world(2, "median", "sharded", 0, 6, tmp_path, ckpt=True)
    single = _single(2, "median", "sharded", 0, 6)
    for a, b in zip(res[0]["params"], single):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def _save_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from consensusml_amd.parallel import dist as D
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    D._INFO = None
    info = D.init_distributed("gloo")
    cfg = _cfg("krum", "sharded", 1, 0, 3)
    cfg.optim.momentum = 0.9
    cfg.ckpt_dir = os.path.join(out_dir, "ckpt")
    cfg.ckpt_every = 3
    tr = ConsensusTrainer(cfg, info=info)
    tr.fit(3, log_every=0)
    torch.save({"params": [p.detach().clone() for p in tr.model.parameters()],
                "master": tr.engine.master.clone()}, os.path.join(out_dir, f"saved{rank}.pt"))
    D.monitored_barrier(30)
    dist.destroy_process_group()


def _load_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from consensusml_amd.parallel import dist as D
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    D._INFO = None
    info = D.init_distributed("gloo")
    cfg = _cfg("krum", "sharded", 1, 0, 3)
    cfg.optim.momentum = 0.9
    tr = ConsensusTrainer(cfg, info=info)
    r = tr.load(os.path.join(out_dir, "ckpt"))
    assert r["resharded"]
    saved = torch.load(os.path.join(out_dir, "saved0.pt"), weights_only=True)
    for a, b in zip(tr.model.parameters(), saved["params"]):
        assert torch.equal(a.detach(), b)
    tr.fit(5, log_every=0)     # keeps training after the re-shard
    torch.save({"params": [p.detach().clone() for p in tr.model.parameters()],
                "step": tr.engine.step_count}, os.path.join(out_dir, f"w{world}_{rank}.pt"))
    D.monitored_barrier(30)
    dist.destroy_process_group()


def test_checkpoint_reshard_world2_to_1_and_4(tmp_path):
    """A sharded checkpoint written by 2 ranks loads at world 1 (this process) and world 4 with
    the parameters and fp32 master unchanged; the consensus table is written next to it."""
    import pandas as pd
    from consensusml_amd.parallel.dist import DistInfo
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    mp.spawn(_save_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    saved = torch.load(tmp_path / "saved0.pt", weights_only=True)
    # consensus table of the checkpoint step: one row per parameter tensor + per-worker rows
    tab = pd.read_csv(tmp_path / "ckpt" / "step_3" / "consensus_table.csv", index_col=0)
    assert {"grad_norm_w0", "grad_norm_w1", "dist_to_agg_w0", "agg_norm"} <= set(tab.columns)
    assert "(selection_count)" in tab.index and len(tab) == len(saved["params"]) + 3
    # world 1
    from consensusml_amd.parallel import dist as D
    D._INFO = None
    cfg = _cfg("krum", "sharded", 1, 0, 3)
    cfg.optim.momentum = 0.9
    tr = ConsensusTrainer(cfg, info=DistInfo(0, 1, 0, torch.device("cpu"), "none"))
    r = tr.load(str(tmp_path / "ckpt"))
    assert r["resharded"] and tr.engine.step_count == 3
    for a, b in zip(tr.model.parameters(), saved["params"]):
        torch.testing.assert_close(a.detach(), b, rtol=0, atol=0)
    # the world-1 master is the full vector: its parameter values equal the saved params
    for p, (n, o, k) in zip(tr.model.parameters(), tr.engine.flat.segments()):
        torch.testing.assert_close(tr.engine.master[o:o + k].view_as(p), p.detach().float())
    # world 4
    mp.spawn(_load_worker, args=(4, _free_port(), str(tmp_path)), nprocs=4, join=True)
    for rk in range(4):
        got = torch.load(tmp_path / f"w4_{rk}.pt", weights_only=True)
        assert got["step"] == 5
        assert all(torch.isfinite(p).all() for p in got["params"])


def test_param_prefetch_bit_identical(tmp_path):
    """Overlapping the sharded parameter all-gather with the next forward (per-module waits)
    gives bit-identical parameters to waiting for it at the end of the step."""
    (tmp_path / "on").mkdir()
    (tmp_path / "off").mkdir()
    a = _run_world(3, "krum", "sharded", 0, 5, tmp_path / "on", prefetch=True)
    b = _run_world(3, "krum", "sharded", 0, 5, tmp_path / "off", prefetch=False)
    for r in range(3):
        for x, y in zip(a[r]["params"], b[r]["params"]):
            assert torch.equal(x, y)


def _log_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from consensusml_amd.parallel import dist as D
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    D._INFO = None
    info = D.init_distributed("gloo", timeout_s=60)
    cfg = _cfg("krum", "sharded", 1, 0, 4)
    cfg.log_path = os.path.join(out_dir, "log.jsonl")
    tr = ConsensusTrainer(cfg, info=info)
    # every step is a log step: the stats all-reduces must run on every rank, not on the
    # logging rank 0 alone (which would mismatch the collectives and hang)
    tr.fit(4, log_every=1)
    tr.close()
    torch.save({"params": [p.detach().clone() for p in tr.model.parameters()]},
               os.path.join(out_dir, f"log{rank}.pt"))
    D.monitored_barrier(30)
    dist.destroy_process_group()


def test_fit_with_log_path_multirank(tmp_path):
    """fit() with a log path and log_every = 1 on 2 sharded ranks completes, rank 0 writes one
    record per step with the recorded statistics, and the replicas stay identical."""
    import json
    mp.spawn(_log_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    recs = [json.loads(l) for l in open(tmp_path / "log.jsonl")]
    assert [r["step"] for r in recs] == [1, 2, 3, 4]
    assert all("worker_grad_norm" in r and len(r["worker_grad_norm"]) == 2 for r in recs)
    a = torch.load(tmp_path / "log0.pt", weights_only=True)["params"]
    b = torch.load(tmp_path / "log1.pt", weights_only=True)["params"]
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("topo,rule,f", [("sharded", "krum", 0), ("allgather", "multi_krum", 1),
                                         ("sharded", "centered_clip", 0)])
def test_early_gram_bit_identical(tmp_path, topo, rule, f):
    """Per-bucket Gram partials computed as each exchange lands (during backward) and summed in
    bucket order give bit-identical parameters to the Gram computed after the last exchange."""
    (tmp_path / "on").mkdir()
    (tmp_path / "off").mkdir()
    a = _run_world(3, rule, topo, f, 5, tmp_path / "on", early_gram=True)
    b = _run_world(3, rule, topo, f, 5, tmp_path / "off", early_gram=False)
    assert a[0]["early_grams"] > 0 and b[0]["early_grams"] == 0
    for r in range(3):
        for x, y in zip(a[r]["params"], b[r]["params"]):
            assert torch.equal(x, y)
