"""Multi-rank engine on one MI355X: R ranks share cuda:0 over a gloo process group (RCCL refuses
two ranks on one device), so the distributed exchange paths -- all-to-all of gradient shards,
fp64 Gram all-reduce, bf16/fp32 parameter all-gather, bucket hooks -- run with the HIP aggregation
and optimizer kernels on the device. R ranks x 1 worker must equal 1 rank x R virtual workers
(same per-worker data), and every rank must hold bit-identical parameters.

The CPU twin of this test is tests/test_dist_gloo.py; the driver's 8-GPU RCCL run uses the same
engine code with backend "nccl".
"""
import os

import pytest
import torch
import torch.multiprocessing as mp

from test_dist_gloo import _cfg, _free_port

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, rule, topo, f, steps, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from consensusml_amd.parallel import dist as D
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    D._INFO = None
    info = D.init_distributed("gloo", device="cuda:0")
    tr = ConsensusTrainer(_cfg(rule, topo, 1, f, steps), info=info)
    tr.fit(steps, log_every=0)
    torch.cuda.synchronize()
    params = [p.detach().cpu().clone() for p in tr.model.parameters()]
    torch.save({"params": params, "sel": tr.engine.sel_counts.cpu().clone()},
               os.path.join(out_dir, f"r{rank}.pt"))
    D.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("topo,rule,world,f", [
    ("sharded", "krum", 2, 0),          # the bench's topology / rule
    ("sharded", "median", 2, 0),
    ("allgather", "multi_krum", 3, 0),
    ("sharded", "trimmed_mean", 3, 1),
    ("allreduce", "mean", 2, 0),        # the bench's all-reduce reference run
])
def test_gpu_ranks_equal_virtual_workers(cuda, tmp_path, topo, rule, world, f):
    from consensusml_amd.parallel.dist import DistInfo
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    steps = 4
    mp.spawn(_worker, args=(world, _free_port(), rule, topo, f, steps, str(tmp_path)),
             nprocs=world, join=True)
    res = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True)
           for r in range(world)]
    for r in range(1, world):
        for a, b in zip(res[0]["params"], res[r]["params"]):
            assert torch.equal(a, b), f"rank {r} diverged from rank 0"
    cfg = _cfg(rule, topo, world, f, steps)
    tr = ConsensusTrainer(cfg, info=DistInfo(0, 1, 0, cuda, "none"))
    tr.fit(steps, log_every=0)
    for a, b in zip(res[0]["params"], tr.model.parameters()):
        torch.testing.assert_close(a, b.detach().cpu(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(res[0]["sel"], tr.engine.sel_counts.cpu())


@pytest.mark.parametrize("topo,rule,world,f", [
    ("allgather", "krum", 3, 1),
    ("sharded", "krum", 4, 1),
    ("sharded", "geomed", 3, 0),
    ("sharded", "bulyan", 7, 1),        # n >= 4f + 3
])
def test_gpu_ranks_robust_rules(cuda, tmp_path, topo, rule, world, f):
    test_gpu_ranks_equal_virtual_workers(cuda, tmp_path, topo, rule, world, f)


def _prefetch_worker(rank, world, port, out_dir, prefetch):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from consensusml_amd.parallel import dist as D
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    D._INFO = None
    info = D.init_distributed("gloo", device="cuda:0")
    cfg = _cfg("krum", "sharded", 1, 0, 5)
    cfg.dtype = "bf16"
    cfg.topology.param_prefetch = prefetch
    tr = ConsensusTrainer(cfg, info=info)
    tr.fit(5, log_every=0)
    torch.cuda.synchronize()
    torch.save({"params": [p.detach().cpu().clone() for p in tr.model.parameters()]},
               os.path.join(out_dir, f"p{int(prefetch)}_{rank}.pt"))
    D.barrier()
    dist.destroy_process_group()


def test_gpu_param_prefetch_bit_identical(cuda, tmp_path):
    """Sharded bf16 parameters all-gathered behind the next forward (per-module waits) are
    bit-identical to the synchronous all-gather, on the GPU kernels."""
    for pf in (True, False):
        mp.spawn(_prefetch_worker, args=(3, _free_port(), str(tmp_path), pf), nprocs=3,
                 join=True)
    for r in range(3):
        a = torch.load(tmp_path / f"p1_{r}.pt", weights_only=True)["params"]
        b = torch.load(tmp_path / f"p0_{r}.pt", weights_only=True)["params"]
        for x, y in zip(a, b):
            assert torch.equal(x, y)


def _gossip_worker(rank, world, port, out_dir, asyn):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from consensusml_amd import TrainConfig
    from consensusml_amd.parallel import dist as D
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    D._INFO = None
    info = D.init_distributed("gloo", device="cuda:0")
    cfg = TrainConfig()
    cfg.model.name = "llama_tiny"
    cfg.model.seq_len = 64
    cfg.dtype = "bf16"
    cfg.batch_per_worker = 4
    cfg.agg.rule = "mean"
    cfg.topology.kind = "gossip"
    cfg.topology.gossip_async = asyn
    cfg.topology.bucket_mb = 1.0
    cfg.optim.name = "adamw"
    cfg.optim.lr = 3e-3
    cfg.optim.weight_decay = 0.01
    cfg.backend = "gloo"
    tr = ConsensusTrainer(cfg, info=info)
    res = tr.fit(8, log_every=0)
    tr.close()
    torch.cuda.synchronize()
    torch.save({"params": [p.detach().float().cpu().clone() for p in tr.model.parameters()],
                "history": res["history"]}, os.path.join(out_dir, f"g{rank}.pt"))
    D.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("asyn", [False, True])
def test_gpu_gossip_ring_llama_tiny(cuda, tmp_path, asyn):
    """Decentralised gossip (synchronous and delayed) with 3 ranks on the GPU: bf16 llama_tiny,
    fused AdamW, ring send/recv + the HIP mixing kernel. Losses stay finite and bounded (the
    synthetic tokens are uniform: the loss sits at ~log(vocab)), and mixing keeps the replicas
    close to each other."""
    world = 3
    mp.spawn(_gossip_worker, args=(world, _free_port(), str(tmp_path), asyn), nprocs=world,
             join=True)
    res = [torch.load(tmp_path / f"g{r}.pt", weights_only=True) for r in range(world)]
    for r in range(world):
        h = res[r]["history"]
        assert all(torch.isfinite(torch.tensor(h))) and max(h) < h[0] + 1.0
    for ps in zip(*[res[r]["params"] for r in range(world)]):
        spread = torch.stack(ps).std(0).max()
        assert spread < 0.05 * max(p.abs().max() for p in ps) + 1e-2
