"""The engine's distributed code path on a 1-rank process group ("loopback").

With ``init_distributed(..., loopback=True)`` and WORLD_SIZE 1 the engine issues every
collective of an N > 1 run -- the bucketed all-to-all of gradient shards polled with
``is_completed()`` from the backward hooks (early Gram), the fp64 Gram all-reduce, the in-place
bf16 parameter all-gather waited per module by the next forward (prefetch), the all-reduce of the
baseline, and the gossip ``batch_isend_irecv`` -- to the rank itself. On a GPU box with backend
``nccl`` that is RCCL executing the N > 1 engine on the lease's one MI355X.

A loopback run must be bit-identical to the same run without a process group (the collectives
are copies and 1-rank sums), and gossip must equal the mixing formula applied to the local
update (the neighbour IS this rank). The CPU twin uses gloo; the GPU test uses nccl = RCCL.
"""
import collections
import json
import os

import pytest
import torch
import torch.multiprocessing as mp

from test_dist_gloo import _cfg

COLLECTIVES = ("all_to_all_single", "all_gather_into_tensor", "all_reduce", "batch_isend_irecv",
               "broadcast")

CASES = [
    # (topology, rule, f, early_gram_eager)
    ("sharded", "krum", 0, True),
    ("sharded", "krum", 0, False),
    ("sharded", "median", 0, False),
    ("allgather", "multi_krum", 0, True),
    ("allreduce", "mean", 0, False),
    ("sharded", "geomed", 0, False),
]
GOSSIP = ["ring", "exp"]


def _count_collectives(dist):
    calls = collections.Counter()
    for name in COLLECTIVES:
        orig = getattr(dist, name)

        def wrap(*a, _o=orig, _n=name, **k):
            calls[_n] += 1
            return _o(*a, **k)
        setattr(dist, name, wrap)
    return calls


def _loopback_worker(_rank, backend, device, dtype, steps, out_path):
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import torch.distributed as dist
    from consensusml_amd.parallel import dist as D
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    D._INFO = None
    info = D.init_distributed(backend, device=device, loopback=True)
    assert info.loopback and info.distributed and dist.get_world_size() == 1
    plain = D.DistInfo(0, 1, 0, info.device, "none")
    calls = _count_collectives(dist)
    dev = info.device
    res = {"backend": dist.get_backend(), "cases": []}
    for topo, rule, f, eager in CASES:
        out = {}
        for name, inf in (("loop", info), ("plain", plain)):
            cfg = _cfg(rule, topo, 1, f, steps)
            cfg.dtype = dtype
            cfg.backend = backend
            calls.clear()
            tr = ConsensusTrainer(cfg, info=inf)
            tr.engine._gram_eager = eager
            tr.fit(steps, log_every=0)
            if dev.type == "cuda":
                torch.cuda.synchronize()
            out[name] = {"params": [p.detach().float().cpu().clone() for p in tr.model.parameters()],
                         "sel": tr.engine.sel_counts.cpu().clone(),
                         "calls": dict(calls), "early_grams": tr.engine.early_grams,
                         "overlap": tr.engine.overlap, "prefetch": tr.engine.param_prefetch}
            tr.close()
        same = all(torch.equal(a, b) for a, b in zip(out["loop"]["params"], out["plain"]["params"]))
        res["cases"].append({"case": [topo, rule, f, eager], "bit_identical": same,
                             "sel_equal": torch.equal(out["loop"]["sel"], out["plain"]["sel"]),
                             "loop_calls": out["loop"]["calls"],
                             "plain_calls": out["plain"]["calls"],
                             "early_grams": out["loop"]["early_grams"],
                             "overlap": out["loop"]["overlap"],
                             "prefetch": out["loop"]["prefetch"]})
    # gossip: one step; the neighbour buffers hold this rank's own updated parameters
    from consensusml_amd.parallel.engine import gossip_peers
    for graph in GOSSIP:
        ms = {}
        for name, inf in (("loop", info), ("plain", plain)):
            cfg = _cfg("mean", "gossip", 1, 0, 1)
            cfg.dtype = dtype
            cfg.backend = backend
            cfg.topology.gossip_graph = graph
            cfg.topology.gossip_chunk_mb = 0.001     # several pipelined chunks
            calls.clear()
            tr = ConsensusTrainer(cfg, info=inf)
            tr.fit(1, log_every=0)
            ms[name] = (tr.engine.master.detach().cpu().clone(),
                        tr.engine.flat.flat_param.detach().float().cpu().clone(), dict(calls))
            tr.close()
        _, _, w, w0 = gossip_peers(graph, 1, 0, 0)
        m_plain = ms["plain"][0]
        nb = ms["plain"][1]                 # bf16 parameters of the local update
        oracle = m_plain + sum(w) * (nb - m_plain)
        err = float((ms["loop"][0] - oracle).abs().max())
        scale = float(oracle.abs().max())
        res["cases"].append({"case": ["gossip", graph], "mix_err": err, "scale": scale,
                             "loop_calls": ms["loop"][2], "plain_calls": ms["plain"][2]})
    # delayed gossip: the end-of-step mix on a side stream, waited per block by the next forward
    # (param_prefetch), must be bit-identical to the same mix waited for at once
    for graph in GOSSIP:
        outs = {}
        for pf in (True, False):
            cfg = _cfg("mean", "gossip", 1, 0, 3)
            cfg.dtype = dtype
            cfg.backend = backend
            cfg.topology.gossip_graph = graph
            cfg.topology.gossip_async = True
            cfg.topology.param_prefetch = pf
            tr = ConsensusTrainer(cfg, info=info)
            tr.fit(3, log_every=0)
            tr.engine.wait_params()
            if dev.type == "cuda":
                torch.cuda.synchronize()
            outs[pf] = ([p.detach().float().cpu().clone() for p in tr.model.parameters()],
                        tr.engine.master.detach().cpu().clone(), tr.engine.param_prefetch)
            tr.close()
        same = (all(torch.equal(a, b) for a, b in zip(outs[True][0], outs[False][0]))
                and torch.equal(outs[True][1], outs[False][1]))
        res["cases"].append({"case": ["gossip_async", graph], "bit_identical": same,
                             "prefetch": outs[True][2]})
    with open(out_path, "w") as fh:
        json.dump(res, fh)
    dist.destroy_process_group()


def _run(tmp_path, backend, device, dtype, steps=3):
    out = str(tmp_path / f"loop_{backend}.json")
    mp.spawn(_loopback_worker, args=(backend, device, dtype, steps, out), nprocs=1, join=True)
    with open(out) as fh:
        return json.load(fh)


def _check(res, backend):
    assert res["backend"] == backend
    for c in res["cases"]:
        if c["case"][0] == "gossip_async":
            assert c["bit_identical"], c
            assert c["prefetch"] == (backend == "nccl"), c   # the side-stream mix: GPU only
            continue
        if c["case"][0] == "gossip":
            assert c["mix_err"] <= 1e-6 * max(c["scale"], 1.0), c
            if backend == "nccl":   # gloo has no self pairs: the engine copies instead
                assert c["loop_calls"].get("batch_isend_irecv", 0) >= 2, c   # >= 2 chunks
            assert not c["plain_calls"], c
            continue
        topo, rule, _, eager = c["case"]
        assert c["bit_identical"] and c["sel_equal"], c
        assert c["overlap"], c
        lc = c["loop_calls"]
        assert not c["plain_calls"], c
        if topo == "sharded":
            # the gradient all-to-all runs on the 1-rank group; the parameter all-gather and the
            # Gram all-reduce are identities at one rank and are skipped (exercised at 2-8 ranks
            # by tests/test_dist_gloo.py, tests/test_dist_gpu.py)
            assert lc.get("all_to_all_single", 0) > 0
            assert lc.get("all_gather_into_tensor", 0) == 0
            assert c["prefetch"]
        if topo == "allgather":
            assert lc.get("all_gather_into_tensor", 0) > 0
        if topo == "allreduce":
            assert lc.get("all_reduce", 0) > 0
        if rule in ("krum", "multi_krum", "geomed") and topo == "sharded":
            assert lc.get("all_reduce", 0) == 0         # the Gram all-reduce: identity at 1 rank
        if eager:
            assert c["early_grams"] > 0


def test_loopback_gloo_cpu(tmp_path):
    _check(_run(tmp_path, "gloo", "cpu", "fp32"), "gloo")


@pytest.mark.gpu
def test_loopback_rccl_gpu(cuda, tmp_path):
    """RCCL (backend nccl) runs the N > 1 engine on the one GPU: all-to-all + early Grams,
    all-reduce baseline, gossip send/recv (the 1-rank identities -- parameter all-gather, Gram
    all-reduce -- are skipped)."""
    _check(_run(tmp_path, "nccl", "cuda:0", "bf16"), "nccl")
