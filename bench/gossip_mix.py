#!/usr/bin/env python3
"""Gossip mixing kernel at Llama-3-8B scale (D = 8.03 B) on one MI355X.

Times ``gossip_mix_k`` -- x <- x + sum_k w_k clip_k(nb_k - x) on the fp32 master with k bf16
neighbour vectors, writing the bf16 parameters in the same pass -- for k = 1 (the ``exp`` graph),
2 (``ring``) and 5 (``exp_all`` at N = 8), plus the clipped ring (a second pass for the
neighbour distances). Bytes moved per call: master read + write (8 B), k neighbour reads (2k B),
bf16 parameter write (2 B) per coordinate; clipping adds a read of the master and the
neighbours. Memory: 32 GB master + 16 GB params + 16 GB per neighbour buffer (k = 5: 128 GB of
the 288 GB HBM3E).

  python bench/gossip_mix.py --json-out gpurun_out/gossip_mix.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

LLAMA3_8B = 8_030_261_248


def timeit(fn, reps: int) -> float:
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--D", type=int, default=LLAMA3_8B)
    ap.add_argument("--k", type=int, nargs="*", default=[1, 2, 5])
    ap.add_argument("--clip-k", type=int, nargs="*", default=[2])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    from consensusml_amd.ops import kernels as K
    dev = torch.device("cuda", 0)
    D = a.D
    g = torch.Generator(device=dev).manual_seed(0)
    master = torch.randn(D, device=dev, generator=g)
    param = master.to(torch.bfloat16)
    kmax = max(a.k + a.clip_k)
    nbrs = [param.clone() for _ in range(kmax)]
    from consensusml_amd.ops.native import lib
    work = torch.empty(lib().gossip_workspace_bytes(D) // 4, dtype=torch.float32, device=dev)
    rows = []
    for k, clip in [(k, 0.0) for k in a.k] + [(k, 1.0) for k in a.clip_k]:
        w = [1.0 / (k + 1)] * k
        ms = timeit(lambda: K.gossip_mix_k(master, nbrs[:k], w, 1.0 / (k + 1), clip,
                                           param_out=param, work=work), a.reps)
        bytes_ = D * (8 + 2 * k + 2) + (D * (4 + 2 * k) if clip > 0 else 0)
        r = {"kernel": "gossip_mix_k", "D": D, "k": k, "clip": clip, "ms": round(ms, 3),
             "bytes": bytes_, "tb_per_s": round(bytes_ / ms / 1e9, 3),
             "graph": {1: "exp", 2: "ring", 5: "exp_all (N=8)"}.get(k, f"k={k}")}
        rows.append(r)
        print(json.dumps(r), flush=True)
    # a copy of the same bytes for scale: the HBM roof this kernel shape can reach
    src = param
    dst = nbrs[0]
    ms = timeit(lambda: dst.copy_(src), a.reps)
    r = {"kernel": "copy_bf16", "D": D, "ms": round(ms, 3), "bytes": 4 * D,
         "tb_per_s": round(4 * D / ms / 1e9, 3)}
    rows.append(r)
    print(json.dumps(r), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as fh:
            for r in rows:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
