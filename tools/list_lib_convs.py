#!/usr/bin/env python3
"""Which convolutions of the ResNet-50 step still run a library (MIOpen / CK) kernel: wraps
torch.ops.aten.convolution_backward / convolution for one training step at the bench's batch and
prints one JSON line per call (which pass, input / weight shapes, stride, output mask)."""
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    from consensusml_amd import TrainConfig
    from consensusml_amd.parallel.dist import DistInfo
    from consensusml_amd.trainer.trainer import ConsensusTrainer
    from consensusml_amd.utils.tuning import configure_miopen
    configure_miopen()
    torch.backends.cudnn.benchmark = True
    calls = collections.Counter()
    ops = torch.ops.aten
    orig_bwd, orig_fwd = ops.convolution_backward, ops.convolution

    class Wrap:
        def __init__(self, f, tag):
            self.f, self.tag = f, tag

        def __call__(self, *a, **k):
            if self.tag == "bwd":
                dy, x, w = a[0], a[1], a[2]
                mask = tuple(bool(m) for m in a[-1])
                key = ("bwd", tuple(x.shape), tuple(w.shape), tuple(a[4]), mask)
            else:
                x, w = a[0], a[1]
                key = ("fwd", tuple(x.shape), tuple(w.shape), tuple(a[3]), None)
            calls[key] += 1
            return self.f(*a, **k)

    cfg = TrainConfig()
    cfg.model.name = "resnet50"
    cfg.batch_per_worker = batch
    cfg.dtype = "bf16"
    cfg.agg.rule = "krum"
    cfg.topology.kind = "sharded"
    dev = torch.device("cuda", 0)
    tr = ConsensusTrainer(cfg, info=DistInfo(0, 1, 0, dev, "none"))
    tr.train_step()
    torch.cuda.synchronize()
    F = torch.nn.functional
    orig_c2d = F.conv2d

    def c2d(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
        st = tuple(stride) if isinstance(stride, (tuple, list)) else (stride, stride)
        calls[("F.conv2d", tuple(x.shape), tuple(w.shape), st, None)] += 1
        return orig_c2d(x, w, b, stride, padding, dilation, groups)

    ops.convolution_backward = Wrap(orig_bwd, "bwd")
    ops.convolution = Wrap(orig_fwd, "fwd")
    F.conv2d = c2d
    try:
        tr.train_step()
        torch.cuda.synchronize()
    finally:
        ops.convolution_backward, ops.convolution = orig_bwd, orig_fwd
        F.conv2d = orig_c2d
    for (tag, xs, ws, st, mask), c in sorted(calls.items()):
        print(json.dumps({"pass": tag, "x": xs, "w": ws, "stride": st, "mask": mask, "calls": c}))


if __name__ == "__main__":
    main()
