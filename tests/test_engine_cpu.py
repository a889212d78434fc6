"""Engine tests on CPU with virtual workers (single process) — SURVEY.md §4.4 items 4-5."""
import copy

import pytest
import torch

from consensusml_amd import TrainConfig
from consensusml_amd.parallel.dist import DistInfo
from consensusml_amd.trainer.trainer import ConsensusTrainer

CPU = DistInfo(0, 1, 0, torch.device("cpu"), "none")


def make_cfg(rule="median", topo="sharded", V=5, f=1, fault="none", byz=(), steps=20, opt="sgd"):
    cfg = TrainConfig()
    cfg.dtype = "fp32"
    cfg.virtual_workers = V
    cfg.agg.rule = rule
    cfg.agg.f = f
    cfg.topology.kind = topo
    cfg.optim.name = opt
    cfg.optim.lr = 0.1 if opt == "sgd" else 0.01
    cfg.batch_per_worker = 32
    cfg.steps = steps
    cfg.model.extra = {"classes": 2}
    cfg.fault.kind = fault
    cfg.fault.ranks = list(byz)
    return cfg


@pytest.mark.parametrize("topo", ["sharded", "allgather"])
@pytest.mark.parametrize("rule", ["median", "trimmed_mean", "krum", "multi_krum", "geomed",
                                  "bulyan"])
def test_robust_rules_survive_sign_flip(topo, rule):
    V = 7
    cfg = make_cfg(rule, topo, V=V, f=1, fault="sign_flip", byz=[3])
    tr = ConsensusTrainer(cfg, info=CPU)
    r = tr.fit(30, log_every=0)
    ev = tr.evaluate()
    assert r["history"][-1] < 0.4, r["history"][-5:]
    assert ev["accuracy"] > 0.85
    if rule in ("krum", "multi_krum"):
        assert r["selection_counts"][3] == 0


def test_mean_breaks_under_sign_flip():
    cfg = make_cfg("mean", "sharded", V=7, f=0, fault="sign_flip", byz=[3])
    tr = ConsensusTrainer(cfg, info=CPU)
    r = tr.fit(30, log_every=0)
    assert r["history"][-1] > 1.0


@pytest.mark.parametrize("topo", ["allreduce", "allgather", "sharded", "gossip"])
def test_mean_topologies_agree(topo):
    """Without faults, every topology with the mean rule is plain data-parallel SGD."""
    ref = ConsensusTrainer(make_cfg("mean", "allreduce", V=4), info=CPU)
    ref.fit(5, log_every=0)
    tr = ConsensusTrainer(make_cfg("mean", topo, V=4), info=CPU)
    tr.fit(5, log_every=0)
    for a, b in zip(ref.model.parameters(), tr.model.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_engine_matches_torch_sgd():
    """mean over V virtual workers == torch.optim.SGD on the averaged gradient."""
    cfg = make_cfg("mean", "sharded", V=3)
    cfg.optim.weight_decay = 0.01
    cfg.optim.nesterov = True
    tr = ConsensusTrainer(cfg, info=CPU)
    ref_model = copy.deepcopy(tr.model)
    opt = torch.optim.SGD(ref_model.parameters(), lr=0.1, momentum=0.9, weight_decay=0.01,
                          nesterov=True)
    gens = [torch.Generator().manual_seed(cfg.seed * 1000 + v) for v in range(3)]
    for _ in range(4):
        opt.zero_grad()
        for v in range(3):
            b = tr.task.make_batch(32, gens[v])
            (tr.task.loss_fn(ref_model, b) / 3).backward()
        opt.step()
        tr.train_step()
    for a, b in zip(ref_model.parameters(), tr.model.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_adam_engine_matches_torch():
    cfg = make_cfg("mean", "allgather", V=2, opt="adamw")
    cfg.optim.weight_decay = 0.05
    tr = ConsensusTrainer(cfg, info=CPU)
    ref_model = copy.deepcopy(tr.model)
    opt = torch.optim.AdamW(ref_model.parameters(), lr=0.01, weight_decay=0.05)
    gens = [torch.Generator().manual_seed(cfg.seed * 1000 + v) for v in range(2)]
    for _ in range(3):
        opt.zero_grad()
        for v in range(2):
            b = tr.task.make_batch(32, gens[v])
            (tr.task.loss_fn(ref_model, b) / 2).backward()
        opt.step()
        tr.train_step()
    for a, b in zip(ref_model.parameters(), tr.model.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("fault", ["gaussian", "scaled", "zero", "nan", "alie", "ipm"])
def test_fault_kinds_run(fault):
    cfg = make_cfg("median", "sharded", V=5, f=1, fault=fault, byz=[0])
    cfg.fault.scale = 5.0
    tr = ConsensusTrainer(cfg, info=CPU)
    r = tr.fit(10, log_every=0)
    assert all(torch.isfinite(torch.tensor(h)) for h in r["history"])


def test_centered_clip_and_gossip_clip_run():
    cfg = make_cfg("centered_clip", "sharded", V=5)
    cfg.agg.tau = 0.5
    r = ConsensusTrainer(cfg, info=CPU).fit(10, log_every=0)
    assert r["history"][-1] < r["history"][0]


def test_result_dict_keys():
    tr = ConsensusTrainer(make_cfg("krum", "sharded", V=5, f=1), info=CPU)
    r = tr.fit(3, log_every=0)
    for k in ["final_model", "history", "seed", "selection_counts", "options_string",
              "samples_per_sec"]:
        assert k in r
    ev = tr.evaluate()
    for k in ["confusion_matrix", "test_error", "tpr", "tnr", "fdr", "for"]:
        assert k in ev


def test_channels_last_resnet_flat_views():
    cfg = make_cfg("median", "sharded", V=3)
    cfg.model.name = "resnet_tiny"
    cfg.model.num_classes = 10
    cfg.model.image_size = 16
    cfg.batch_per_worker = 2
    tr = ConsensusTrainer(cfg, info=CPU)
    conv = tr.model.conv1.weight
    assert conv.is_contiguous(memory_format=torch.channels_last)
    loss = tr.train_step()
    assert torch.isfinite(loss)
    idx = [i for i, p in enumerate(tr.engine.flat.params) if p is conv][0]
    gview = tr.engine.flat.grad_views(0)[idx]
    assert gview.is_contiguous(memory_format=torch.channels_last)
    assert gview.abs().sum() > 0
    # every parameter lives inside the flat buffer
    fp = tr.engine.flat.flat_param
    lo, hi = fp.data_ptr(), fp.data_ptr() + fp.numel() * fp.element_size()
    for p in tr.model.parameters():
        assert lo <= p.data_ptr() < hi


def test_adam_l2_vs_adamw_cpu():
    """'adam' with weight decay is torch.optim.Adam (L2 term in the gradient), 'adamw' the
    decoupled form; both match torch.optim on the CPU path of the fused kernel."""
    from consensusml_amd.ops import kernels as K
    torch.manual_seed(0)
    D = 257
    for kind, topt in (("adam", torch.optim.Adam), ("adamw", torch.optim.AdamW)):
        p0 = torch.randn(D)
        master = p0.clone()
        s1, s2 = torch.zeros(D), torch.zeros(D)
        ref = torch.nn.Parameter(p0.clone())
        o = topt([ref], lr=1e-2, weight_decay=0.1, eps=1e-8)
        for step in range(1, 4):
            g = torch.randn(D)
            K.agg_update(g[None], combine="weighted", n=1,
                         opt=K.OptArgs(kind=kind, lr=1e-2, weight_decay=0.1, step=step),
                         master=master, s1=s1, s2=s2)
            ref.grad = g.clone()
            o.step()
        torch.testing.assert_close(master, ref.detach(), rtol=1e-5, atol=1e-6)


def test_jsonl_step_log_has_consensus_stats(tmp_path):
    """JSONL step records carry selection counts, weights, per-worker gradient norms,
    distances to the aggregate and Krum scores."""
    import json
    cfg = make_cfg("krum", "sharded", V=5, f=1, fault="sign_flip", byz=[2])
    cfg.log_path = str(tmp_path / "log.jsonl")
    tr = ConsensusTrainer(cfg, info=CPU)
    tr.fit(4, log_every=2)
    tr.close()
    recs = [json.loads(l) for l in open(cfg.log_path)]
    assert [r["step"] for r in recs] == [2, 4]
    for r in recs:
        assert len(r["selection_counts"]) == 5 and len(r["weights"]) == 5
        assert len(r["worker_grad_norm"]) == 5 and len(r["worker_dist_to_aggregate"]) == 5
        assert len(r["krum_scores"]) == 5 and r["aggregate_grad_norm"] > 0
        # the sign-flipped worker (x10) has the largest gradient norm and is never selected
        assert max(range(5), key=lambda i: r["worker_grad_norm"][i]) == 2
        assert r["weights"][2] == 0.0


def test_single_pass_center_equals_two_pass_cpu():
    """One Gram pass centered at the previous step's medoid selects what the two-pass scheme
    selects (CPU reference path), including after the center row turns non-finite."""
    import torch
    from consensusml_amd import TrainConfig
    from consensusml_amd.parallel.dist import DistInfo
    from consensusml_amd.parallel.engine import ConsensusEngine

    def eng(two):
        torch.manual_seed(0)
        cfg = TrainConfig()
        cfg.virtual_workers = 8
        cfg.agg.rule = "multi_krum"
        cfg.agg.f = 2
        cfg.agg.gram_two_pass = two
        cfg.topology.kind = "sharded"
        cfg.topology.bucket_mb = 0.01
        cfg.optim.lr = 0.0
        return ConsensusEngine(torch.nn.Linear(64, 64), cfg, DistInfo())

    one, two = eng(False), eng(True)
    g = torch.Generator().manual_seed(5)
    for step in range(4):
        base = torch.randn(one.flat.total, generator=g)
        X = base + 0.01 * torch.randn(8, one.flat.total, generator=g)
        X[6:] = base + 0.5 * torch.randn(2, one.flat.total, generator=g)
        if step == 3:
            X[int(one.center[0])] = float("nan")
        for e in (one, two):
            e.zero_grad()
            e.flat.flat_grad.copy_(X.to(e.flat.flat_grad.dtype))
            e._flushed = {b.index for b in e.flat.buckets}
            e.step()
        assert torch.equal(one.w, two.w), step
        assert one.have_center
