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
