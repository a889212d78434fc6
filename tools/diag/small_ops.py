"""Which Python lines launch the PyTorch elementwise / copy / reduce kernels of a ResNet-50
training step (bench.py's Krum/sharded step at one batch): torch.profiler CPU events with
stacks, grouped by (op, first consensusml_amd / bench frame)."""
import argparse
import collections
import sys

import torch

sys.path.insert(0, ".")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    from consensusml_amd import TrainConfig
    from consensusml_amd.parallel.dist import DistInfo
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = TrainConfig()
    cfg.model.name = "resnet50"
    cfg.batch_per_worker = a.batch
    cfg.dtype = "bf16"
    cfg.agg.rule = "krum"
    cfg.agg.f = 0
    cfg.topology.kind = "sharded"
    cfg.optim.name = "sgd"
    cfg.optim.lr = 0.1
    cfg.optim.momentum = 0.9
    tr = ConsensusTrainer(cfg, info=DistInfo(device=dev))
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    batch = tr.task.make_batch(a.batch, gen)
    model, eng = tr.model, tr.engine

    def step():
        eng.zero_grad()
        tr.task.loss_fn(model, batch).backward()
        eng.step()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    groups = collections.Counter()
    keep = {"copy_", "_to_copy", "mul", "add", "mean", "sum", "fill_", "cat", "clamp",
            "remainder", "div", "sub", "mv", "zero_", "arange", "ne", "eq", "abs", "lt", "max",
            "all", "gt", "bitwise_and", "add_", "mul_", "addmm", "mm", "clamp_min", "argmax",
            "div_", "sub_", "copy", "clone", "contiguous", "index", "where", "neg", "sqrt"}

    class Rec(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = func.overloadpacket.__name__
            if name in keep:
                fr = [f for f in traceback.extract_stack()
                      if ("consensusml_amd" in f.filename or "bench" in f.filename
                          or "small_ops" in f.filename) and "site-packages" not in f.filename
                      and f.name != "__torch_dispatch__"]
                where = " < ".join(f"{f.filename.split('/')[-1]}:{f.lineno} {f.name}"
                                   for f in fr[::-1][:3]) if fr else "?"
                groups[(name, where)] += 1
            return func(*args, **(kwargs or {}))
    with Rec():
        step()
        torch.cuda.synchronize()
    for (name, where), n in sorted(groups.items(), key=lambda kv: -kv[1]):
        print(f"{n:4d}  {name:22s} {where}")


if __name__ == "__main__":
    main()
