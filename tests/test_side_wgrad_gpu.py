"""Weight gradients on a side HIP stream (ops.side, PerfPolicy.side_wgrad): the same kernels on
the same inputs. Three ResNet-50 training steps through the consensus engine with and without the
side stream agree as closely as two runs without it (MIOpen's split-K weight-gradient kernels for
the library shapes sum with atomics, so even those two need not be bit-identical; a race would
show as a far larger difference); and a plain autograd backward outside the engine (not armed)
never uses the side stream."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(cuda, side_on: bool, steps: int = 3):
    from consensusml_amd import TrainConfig, perf
    from consensusml_amd.parallel.dist import DistInfo
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    cfg = TrainConfig()
    cfg.model.name = "resnet50"
    cfg.model.num_classes = 10
    cfg.model.image_size = 64
    cfg.batch_per_worker = 16
    cfg.virtual_workers = 2
    cfg.agg.rule = "krum"
    cfg.agg.f = 0
    cfg.topology.kind = "sharded"
    cfg.optim.name = "sgd"
    cfg.optim.lr = 0.05
    cfg.seed = 3
    pol = perf.policy().replace(side_wgrad=side_on)
    with perf.use_policy(pol):
        tr = ConsensusTrainer(cfg, info=DistInfo(0, 1, 0, cuda, "none"))
        losses = [float(tr.train_step()) for _ in range(steps)]
        torch.cuda.synchronize()
        params = tr.engine.flat.flat_param.clone()
        tr.close()
    return losses, params


def test_side_wgrad_matches_inline(cuda):
    from consensusml_amd.ops import side
    l0, p0 = _train(cuda, False)
    l0b, p0b = _train(cuda, False)
    l1, p1 = _train(cuda, True)
    assert side._S.armed is None   # step() disarmed it
    floor = float((p0b.float() - p0.float()).norm())
    diff = float((p1.float() - p0.float()).norm())
    scale = float(p0.float().norm())
    assert l1[0] == l0[0]          # the first step's loss precedes any weight gradient
    assert diff <= max(4 * floor, 1e-5 * scale), (diff, floor, scale)
    for a, b, c in zip(l0, l0b, l1):
        assert abs(c - a) <= max(4 * abs(b - a), 1e-5 * abs(a)), (l0, l0b, l1)


def test_side_not_armed_outside_engine(cuda):
    from consensusml_amd import perf
    from consensusml_amd.models import resnet50
    from consensusml_amd.ops import side
    m = resnet50(10).to(cuda, torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(8, 3, 64, 64, device=cuda).bfloat16().contiguous(
        memory_format=torch.channels_last)
    with perf.use_policy(perf.policy().replace(side_wgrad=True)):
        m(x).float().sum().backward()
    assert side._S.used is False and side._S.armed is None
    assert all(p.grad is not None and torch.isfinite(p.grad.float()).all() for p in m.parameters())
