#!/usr/bin/env python3
"""Identity-block backward fusion A/B per ResNet-50 stage (PerfPolicy.fused_bn3_bwd).

For each stage shape (planes 64/128/256/512 at 56/28/14/7 px, batch 2048) a chain of three
identity Bottlenecks runs forward + backward with the fused tail on and off; ms per chain
iteration (median of 5 after warm-up). One JSON line per stage.

  python bench/bwd_fusion.py --batch 2048
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--blocks", type=int, default=3)
    ap.add_argument("--stages", default="64:56,128:28,256:14,512:7")
    a = ap.parse_args()
    from consensusml_amd.models.resnet import Bottleneck
    from consensusml_amd.ops.bn import ResidualLink
    from consensusml_amd.utils.tuning import configure_miopen
    configure_miopen()
    dev = torch.device("cuda:0")
    from consensusml_amd import perf
    for item in a.stages.split(","):
        planes, H = (int(v) for v in item.split(":"))
        torch.manual_seed(0)
        m = torch.nn.Sequential(*[Bottleneck(planes * 4, planes) for _ in range(a.blocks)])
        m = m.to(device=dev, dtype=torch.bfloat16, memory_format=torch.channels_last).train()
        x = torch.randn(a.batch, planes * 4, H, H, device=dev).bfloat16().contiguous(
            memory_format=torch.channels_last).requires_grad_(True)
        gy = torch.randn_like(x)
        res = {}
        for flag in (False, True, False, True):
            # the A/B covers every stage
            perf.set_policy(perf.policy().replace(fused_bn3_bwd=flag,
                                                  fused_bn3_bwd_max_planes=4096))
            ts = []
            for it in range(8):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                # as inside the network: the chain input carries its producer's residual link
                xin = x.view_as(x)
                xin._cml_link = ResidualLink()
                y = m(xin)
                y.backward(gy)
                e.record()
                torch.cuda.synchronize()
                if it >= 3:
                    ts.append(s.elapsed_time(e))
            ts.sort()
            res.setdefault(flag, []).append(ts[len(ts) // 2])
            x.grad = None
            m.zero_grad(set_to_none=True)
        off, on = min(res[False]), min(res[True])
        print(json.dumps({"planes": planes, "hw": H, "batch": a.batch, "blocks": a.blocks,
                          "unfused_ms": round(off, 3), "fused_ms": round(on, 3),
                          "saved_ms_per_block": round((off - on) / a.blocks, 3)}), flush=True)
        del m, x, gy
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
