"""Batched virtual workers (ops/worker_grads.py, ConsensusEngine.worker_batch): the V micro-batches
of a BERT step as ONE forward / backward with per-worker parameter gradients written straight
into the engine's gradient rows, against the sequential loop (one forward / backward per worker,
copy-on-ready capture) from the same initial weights and data.

Activations are per token / per sequence in BERT, so every per-worker gradient is the same math;
the two paths differ only in GEMM shapes (M = V x tokens vs tokens) and reduction order, hence a
bf16-rounding tolerance per gradient row rather than bit equality."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _trainer(batched: bool, V: int, rule: str, seq: int, batch: int, lr: float):
    from consensusml_amd import TrainConfig, perf
    from consensusml_amd.parallel.dist import DistInfo
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    cfg = TrainConfig()
    cfg.model.name = "bert_tiny"
    cfg.model.seq_len = seq
    cfg.batch_per_worker = batch
    cfg.virtual_workers = V
    cfg.agg.rule = rule
    cfg.agg.f = 1 if rule in ("krum", "multi_krum") else 0
    cfg.topology.kind = "sharded"
    cfg.optim.name = "adamw"
    cfg.optim.lr = lr
    cfg.seed = 5
    cfg.dtype = "bf16"
    pol = perf.policy().replace(batched_workers=batched)
    with perf.use_policy(pol):
        tr = ConsensusTrainer(cfg, info=DistInfo(0, 1, 0, torch.device("cuda", 0), "none"))
    return tr, pol


def _rel_rows(a, b):
    return ((a.float() - b.float()).norm(dim=1) / b.float().norm(dim=1).clamp_min(1e-12))


@pytest.mark.parametrize("V,seq,batch", [(4, 32, 2), (8, 64, 1)])
def test_batched_grads_match_sequential(cuda, V, seq, batch):
    from consensusml_amd import perf
    out = {}
    for batched in (False, True):
        tr, pol = _trainer(batched, V, "geomed", seq, batch, lr=0.0)
        with perf.use_policy(pol):
            loss = tr.train_step()
        torch.cuda.synchronize()
        out[batched] = (float(loss), tr.engine.flat.flat_grad.clone())
        tr.close()
    (l0, g0), (l1, g1) = out[False], out[True]
    assert abs(l0 - l1) <= 1e-3 * abs(l0)
    assert g0.shape == g1.shape and g0.shape[0] == V
    rel = _rel_rows(g1, g0)
    assert float(rel.max()) < 2e-2, rel.tolist()
    # every parameter's gradient block is produced (nothing left as stale / zero rows)
    assert bool((g1.float().norm(dim=1) > 0).all())


def test_batched_training_tracks_sequential(cuda):
    """Five robust (Krum) steps: same loss trajectory and selected rows as the sequential loop."""
    from consensusml_amd import perf
    res = {}
    for batched in (False, True):
        tr, pol = _trainer(batched, 6, "krum", 32, 2, lr=1e-3)
        with perf.use_policy(pol):
            losses = [float(tr.train_step()) for _ in range(5)]
        torch.cuda.synchronize()
        res[batched] = (losses, tr.engine.flat.flat_param.float().clone(),
                        tr.engine.sel_counts.cpu().clone())
        tr.close()
    (la, pa, sa), (lb, pb, sb) = res[False], res[True]
    for x, y in zip(la, lb):
        assert abs(x - y) <= 5e-3 * abs(x)
    assert float((pb - pa).norm() / pa.norm()) < 5e-3
    assert torch.equal(sa, sb)


def test_batched_rejects_unsupported_param(cuda):
    """A parameter whose op has no per-worker path must fail loudly, not be silently summed."""
    from consensusml_amd.ops import worker_grads as WG
    tr, _ = _trainer(True, 2, "mean", 32, 1, lr=0.0)
    e = tr.engine
    e.zero_grad()
    extra = tr.model.head.weight
    with pytest.raises(RuntimeError, match="no per-worker gradient path"):
        with e.worker_batch():
            assert WG.current() is not None
            # a plain autograd use of a parameter bypasses the per-worker ops
            (extra.float().sum() * 1.0).backward()
    tr.close()
