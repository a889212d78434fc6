"""Direct gradients (TopologyConfig.direct_grads): with one worker per rank the ops that have a
per-worker gradient path (ops/worker_grads.py: Llama's bias-free projections and output head,
BERT's linears / fused FFN / embedding, the norms) write their parameter gradients straight into
the engine's flat gradient row during backward; the AccumulateGrad hooks still fire (without a
gradient) and drive the bucket flushes. Against the copy-on-ready capture from the same weights
and data: the LinearNB gradients are the same GEMM into a different buffer (bit-identical), the
norm / embedding paths reduce in another order (bf16-rounding tolerance)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _trainer(model: str, direct: bool, lr: float, rule: str = "mean"):
    from consensusml_amd import TrainConfig
    from consensusml_amd.parallel.dist import DistInfo
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    cfg = TrainConfig()
    cfg.model.name = model
    cfg.model.seq_len = 64
    cfg.batch_per_worker = 2
    cfg.virtual_workers = 1
    cfg.agg.rule = rule
    cfg.topology.kind = "sharded"
    cfg.topology.bucket_mb = 0.25       # several buckets: flushes interleave with backward
    cfg.topology.direct_grads = direct
    cfg.optim.name = "adamw"
    cfg.optim.lr = lr
    cfg.seed = 11
    cfg.dtype = "bf16"
    return ConsensusTrainer(cfg, info=DistInfo(0, 1, 0, torch.device("cuda", 0), "none"))


def _count_direct(monkeypatch):
    from consensusml_amd.ops import worker_grads as WG
    calls = {"n": 0}
    orig = WG.WorkerGrads.out

    def out(self, p):
        calls["n"] += 1
        return orig(self, p)
    monkeypatch.setattr(WG.WorkerGrads, "out", out)
    return calls


@pytest.mark.parametrize("model", ["llama_tiny", "bert_tiny"])
def test_direct_grads_match_capture(cuda, model, monkeypatch):
    calls = _count_direct(monkeypatch)
    out = {}
    for direct in (False, True):
        tr = _trainer(model, direct, lr=0.0)
        n0 = calls["n"]
        loss = tr.train_step()
        torch.cuda.synchronize()
        out[direct] = (float(loss), tr.engine.flat.flat_grad[0].clone(), calls["n"] - n0)
        fl = tr.engine.flat
        names = fl.param_names()
        offs = [fl.param_offset[i] for i in range(len(fl.params))]
        shapes = [p.numel() for p in fl.params]
        tr.close()
    (l0, g0, c0), (l1, g1, c1) = out[False], out[True]
    assert c0 == 0 and c1 > 0                      # the direct path really ran
    assert abs(l0 - l1) <= 1e-6 * max(1.0, abs(l0))
    for name, off, n in zip(names, offs, shapes):
        a, b = g0[off:off + n].float(), g1[off:off + n].float()
        assert b.norm() > 0, name                  # produced, not a zero / stale row
        rel = float((a - b).norm() / a.norm().clamp_min(1e-12))
        assert rel < 1e-2, (name, rel)


def test_direct_grads_llama_projections_bitwise(cuda):
    """The bias-free projections and the output head: the same GEMM written in place."""
    out = {}
    for direct in (False, True):
        tr = _trainer("llama_tiny", direct, lr=0.0)
        tr.train_step()
        torch.cuda.synchronize()
        fl = tr.engine.flat
        out[direct] = {n: fl.flat_grad[0, fl.param_offset[i]:fl.param_offset[i] + p.numel()].clone()
                       for i, (n, p) in enumerate(zip(fl.param_names(), fl.params))
                       if p.dim() == 2 and "tok" not in n}
        tr.close()
    assert out[False].keys() == out[True].keys() and out[False]
    for n in out[False]:
        assert torch.equal(out[False][n], out[True][n]), n


def test_direct_grads_training_tracks_capture(cuda):
    """Five AdamW steps: the same loss trajectory and parameters."""
    res = {}
    for direct in (False, True):
        tr = _trainer("llama_tiny", direct, lr=1e-3)
        losses = [float(tr.train_step()) for _ in range(5)]
        torch.cuda.synchronize()
        res[direct] = (losses, tr.engine.flat.flat_param.float().clone())
        tr.close()
    (la, pa), (lb, pb) = res[False], res[True]
    for x, y in zip(la, lb):
        assert abs(x - y) <= 5e-3 * abs(x)
    assert float((pb - pa).norm() / pa.norm()) < 5e-3
