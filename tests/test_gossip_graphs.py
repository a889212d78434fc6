"""Gossip communication graphs on 4 gloo ranks (CPU; GPU twin in tests/test_dist_gpu.py).

Each rank starts from its own perturbed replica, lr = 0 (pure mixing), and the consensus
distance sqrt(mean_i ||x_i - mean x||^2) is measured after every step. At equal bytes sent
per rank (ring: 2 vectors per step, exp: 1, exp_all: 3 at N = 4) the exponential graphs must
contract faster than the ring; exp reaches the average after log2 N = 2 steps (up to the bf16
rounding of the exchanged parameters). Delayed (async) gossip on the exp graph must resume from
a checkpoint bit-identically to an uninterrupted run.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

BYTES_PER_STEP = {"ring": 2, "exp": 1, "exp_all": 3}   # parameter vectors sent per rank (N = 4)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(graph, asyn=False, dtype="bf16"):
    from consensusml_amd import TrainConfig
    cfg = TrainConfig()
    cfg.dtype = dtype
    cfg.agg.rule = "mean"
    cfg.topology.kind = "gossip"
    cfg.topology.gossip_graph = graph
    cfg.topology.gossip_async = asyn
    cfg.topology.gossip_chunk_mb = 0.001          # several exchange chunks even for the MLP
    cfg.optim.lr = 0.0
    cfg.optim.momentum = 0.0
    cfg.batch_per_worker = 8
    cfg.model.extra = {"classes": 2}
    cfg.backend = "gloo"
    return cfg


def _consensus(master, world):
    import torch.distributed as dist
    xs = [torch.empty_like(master) for _ in range(world)]
    dist.all_gather(xs, master)
    X = torch.stack(xs).double()
    return float(((X - X.mean(0)) ** 2).sum(1).mean().sqrt())


def _contract_worker(rank, world, port, out_dir, graph, device):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from consensusml_amd.parallel import dist as D
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    D._INFO = None
    info = D.init_distributed("gloo", device=device, timeout_s=120)
    tr = ConsensusTrainer(_cfg(graph), info=info)
    e = tr.engine
    g = torch.Generator().manual_seed(100 + rank)
    e.master.add_(torch.randn(e.master.shape, generator=g).to(e.master.device))
    e.flat.flat_param.copy_(e.master.to(e.flat.flat_param.dtype))
    dist_cpu = lambda: _consensus(e.master.detach().cpu(), world)   # noqa: E731
    d = [dist_cpu()]
    for _ in range(4):
        tr.train_step()
        d.append(dist_cpu())
    torch.save({"d": d}, os.path.join(out_dir, f"{graph}_{rank}.pt"))
    D.monitored_barrier(60)
    dist.destroy_process_group()


def run_contraction(tmp_path, device=None):
    out = {}
    for graph in ("ring", "exp", "exp_all"):
        mp.spawn(_contract_worker, args=(4, _free_port(), str(tmp_path), graph, device),
                 nprocs=4, join=True)
        out[graph] = torch.load(tmp_path / f"{graph}_0.pt", weights_only=True)["d"]
    return out


def check_contraction(d):
    d0 = d["ring"][0]
    assert abs(d["exp"][0] - d0) < 1e-9 and abs(d["exp_all"][0] - d0) < 1e-9
    # ring at N = 4: the mixing matrix's second eigenvalue is 1/3
    assert d["ring"][1] < 0.4 * d0
    # exp: exact average after 2 steps (bf16 rounding of the received parameters remains)
    assert d["exp"][2] < 0.01 * d0
    # exp_all at N = 4 talks to all 3 peers: the average after one step
    assert d["exp_all"][1] < 0.01 * d0
    # equal bytes per rank: 4 vectors = 2 ring steps = 4 exp steps; 6 = 3 ring = 2 exp_all
    assert d["exp"][4] < 0.1 * d["ring"][2]
    assert d["exp_all"][2] < 0.1 * d["ring"][3]


def test_gossip_graph_contraction_gloo(tmp_path):
    check_contraction(run_contraction(tmp_path))


def _resume_worker(rank, world, port, out_dir, mode, graph):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from consensusml_amd.parallel import dist as D
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    D._INFO = None
    info = D.init_distributed("gloo", timeout_s=120)
    cfg = _cfg(graph, asyn=True, dtype="fp32")
    cfg.optim.lr = 0.05
    cfg.optim.momentum = 0.9
    cfg.ckpt_dir = os.path.join(out_dir, f"ckpt_{mode}")
    tr = ConsensusTrainer(cfg, info=info)
    if mode == "resume":
        tr.fit(3, log_every=0)
        tr.save()
        tr.close()
        tr = ConsensusTrainer(cfg, info=info)
        tr.load(cfg.ckpt_dir)
    tr.fit(6, log_every=0)
    tr.close()
    torch.save({"params": [p.detach().clone() for p in tr.model.parameters()]},
               os.path.join(out_dir, f"{mode}_{rank}.pt"))
    D.monitored_barrier(60)
    dist.destroy_process_group()


@pytest.mark.parametrize("graph", ["exp", "exp_all"])
def test_delayed_gossip_resume_bit_identical(tmp_path, graph):
    for mode in ("straight", "resume"):
        mp.spawn(_resume_worker, args=(4, _free_port(), str(tmp_path), mode, graph), nprocs=4,
                 join=True)
    for r in range(4):
        a = torch.load(tmp_path / f"straight_{r}.pt", weights_only=True)["params"]
        b = torch.load(tmp_path / f"resume_{r}.pt", weights_only=True)["params"]
        for x, y in zip(a, b):
            assert torch.equal(x, y)
