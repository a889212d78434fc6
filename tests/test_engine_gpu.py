"""Virtual-worker engine tests on one MI355X: n = 8 workers as
micro-batches, every rule / topology through the HIP kernels, Byzantine workers injected."""
import copy

import pytest
import torch

from consensusml_amd import TrainConfig
from consensusml_amd.parallel.dist import DistInfo
from consensusml_amd.trainer.trainer import ConsensusTrainer

pytestmark = pytest.mark.gpu


def _cfg(rule, topo="sharded", V=8, f=2, fault="none", byz=(), model="mlp", dtype="bf16",
         opt="sgd", lr=0.05):
    cfg = TrainConfig()
    cfg.dtype = dtype
    cfg.virtual_workers = V
    cfg.agg.rule = rule
    cfg.agg.f = f
    cfg.topology.kind = topo
    cfg.optim.name = opt
    cfg.optim.lr = lr
    cfg.batch_per_worker = 64
    cfg.model.name = model
    cfg.model.extra = {"classes": 2}
    cfg.fault.kind = fault
    cfg.fault.ranks = list(byz)
    return cfg


def _info(dev):
    return DistInfo(0, 1, 0, dev, "none")


@pytest.mark.parametrize("rule", ["median", "trimmed_mean", "krum", "multi_krum", "geomed",
                                  "bulyan"])
def test_gpu_robust_rules_survive_sign_flip(cuda, rule):
    f = 1 if rule == "bulyan" else 2
    cfg = _cfg(rule, f=f, fault="sign_flip", byz=[1, 6] if rule != "bulyan" else [6])
    if rule == "bulyan":
        cfg.virtual_workers = 8
    tr = ConsensusTrainer(cfg, info=_info(cuda))
    r = tr.fit(60, log_every=0)
    assert r["history"][-1] < 0.45, (rule, r["history"][-5:])
    if rule in ("krum", "multi_krum"):
        sc = r["selection_counts"]
        assert sc[1] == 0 and sc[6] == 0


def test_gpu_mean_diverges_under_attack(cuda):
    tr = ConsensusTrainer(_cfg("mean", f=0, fault="sign_flip", byz=[1, 6]), info=_info(cuda))
    r = tr.fit(40, log_every=0)
    assert r["history"][-1] > 0.69


@pytest.mark.parametrize("topo", ["allgather", "sharded", "allreduce", "gossip"])
def test_gpu_topologies_match_cpu_reference(cuda, topo):
    """fp32 mean over 4 virtual workers: GPU kernels == CPU reference path, same data."""
    cfg = _cfg("mean", topo, V=4, f=0, dtype="fp32")
    g = ConsensusTrainer(cfg, info=_info(cuda))
    c = ConsensusTrainer(copy.deepcopy(cfg), info=_info(torch.device("cpu")))
    c.model.load_state_dict({k: v.cpu() for k, v in g.model.state_dict().items()})
    c.engine.master.copy_(g.engine.master.cpu())
    # identical batches: feed the GPU trainer the CPU batches
    for _ in range(3):
        batches = [c.task.make_batch(64, gen) for gen in c.gens]
        for tr, dev in ((c, "cpu"), (g, cuda)):
            tr.engine.zero_grad()
            for v, (x, y) in enumerate(batches):
                tr.engine.bind_worker(v)
                tr.task.loss_fn(tr.model, (x.to(dev), y.to(dev))).backward()
            tr.engine.step()
    for a, b in zip(c.model.parameters(), g.model.parameters()):
        torch.testing.assert_close(a, b.cpu(), rtol=2e-4, atol=2e-5)


@pytest.mark.parametrize("model,rule,topo,opt", [
    ("resnet_tiny", "krum", "sharded", "sgd"),
    ("bert_tiny", "geomed", "sharded", "adamw"),
    ("llama_tiny", "centered_clip", "allgather", "adamw"),
    ("llama_tiny", "mean", "gossip", "adamw"),
])
def test_gpu_model_families(cuda, model, rule, topo, opt):
    # resnet_tiny (width 8) in bf16 has ~33 % gradient error vs fp32 on PyTorch's own bf16 ops
    # too (tools/diag/tiny_grad.py), so SGD at lr 0.05 / batch 4 follows a noise-driven path: the
    # check is that every family trains through the engine without diverging
    cfg = _cfg(rule, topo, V=4, f=1, model=model, opt=opt, lr=1e-3 if opt == "adamw" else 0.01)
    cfg.model.num_classes = 10
    cfg.model.image_size = 32
    cfg.model.seq_len = 32
    cfg.batch_per_worker = 4
    tr = ConsensusTrainer(cfg, info=_info(cuda))
    r = tr.fit(6, log_every=0)
    assert all(h == h for h in r["history"])
    assert r["history"][-1] < r["history"][0] + 0.5


def test_gpu_checkpoint_roundtrip(cuda, tmp_path):
    cfg = _cfg("krum", V=5, f=1, opt="adamw", lr=1e-3)
    cfg.ckpt_dir = str(tmp_path / "ck")
    a = ConsensusTrainer(cfg, info=_info(cuda))
    a.fit(4, log_every=0)
    a.save()
    a.fit(8, log_every=0)
    b = ConsensusTrainer(cfg, info=_info(cuda))
    b.load(cfg.ckpt_dir)
    b.fit(8, log_every=0)
    for x, y in zip(a.model.parameters(), b.model.parameters()):
        torch.testing.assert_close(x, y)


@pytest.mark.parametrize("optim", ["adamw", "sgd"])
def test_gossip_early_update_matches_step_update(cuda, optim):
    """Gossip with one local worker: per-bucket optimizer steps launched from the backward hooks
    on a side stream give the same parameters as the single update in step()."""
    from consensusml_amd import TrainConfig
    from consensusml_amd.parallel.dist import DistInfo
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    res = []
    for early in (True, False):
        cfg = TrainConfig()
        cfg.model.name = "llama_tiny"
        cfg.model.seq_len = 32
        cfg.batch_per_worker = 2
        cfg.agg.rule = "mean"
        cfg.topology.kind = "gossip"
        cfg.topology.bucket_mb = 0.05      # several buckets
        cfg.topology.early_update = early
        cfg.optim.name = optim
        cfg.optim.lr = 1e-3
        tr = ConsensusTrainer(cfg, info=DistInfo(0, 1, 0, cuda, "none"))
        assert tr.engine.early_update == early
        for _ in range(3):
            tr.train_step()
        torch.cuda.synchronize()
        res.append(torch.cat([p.detach().float().flatten() for p in tr.model.parameters()]))
        tr.close()
    torch.testing.assert_close(res[0], res[1], rtol=0, atol=0)
