#!/usr/bin/env python3
"""Per-shape timing of ResNet-50's convolutions on one MI355X (batch B, bf16, NHWC):
MIOpen (find mode, naive solvers skipped) forward / backward-data / backward-weight vs the
equivalent GEMM formulations for 1x1 stride-1 convolutions (hipBLASLt via torch.mm; weight
gradient also as a split-K batched GEMM). One JSON line per conv shape with achieved TFLOP/s, so
the model can pick the fastest formulation per shape.

  python bench/conv_shapes.py --batch 512 --json-out gpurun_out/conv_shapes.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def resnet50_convs(B: int):
    """(name, N, Cin, H, W, Cout, k, stride, count) for every distinct conv of ResNet-50 v1.5."""
    out = [("stem", B, 3, 224, 224, 64, 7, 2, 1)]
    cin, hw = 64, 56
    for li, (planes, blocks, stride) in enumerate([(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]):
        for b in range(blocks):
            s = stride if b == 0 else 1
            out.append((f"l{li+1}b{b}_conv1", B, cin, hw, hw, planes, 1, 1, 1))
            out.append((f"l{li+1}b{b}_conv2", B, planes, hw, hw, planes, 3, s, 1))
            ohw = hw // s
            out.append((f"l{li+1}b{b}_conv3", B, planes, ohw, ohw, planes * 4, 1, 1, 1))
            if b == 0:
                out.append((f"l{li+1}b{b}_down", B, cin, hw, hw, planes * 4, 1, s, 1))
            cin, hw = planes * 4, ohw
    # merge identical shapes
    merged = {}
    for name, N, C, H, W, K, k, s, c in out:
        key = (N, C, H, W, K, k, s)
        if key in merged:
            merged[key][1] += c
        else:
            merged[key] = [name, c]
    return [(v[0], *k, v[1]) for k, v in merged.items()]


def timeit(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    from consensusml_amd.utils.tuning import configure_miopen
    configure_miopen()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    total = {"miopen": 0.0, "best": 0.0}
    for name, N, C, H, W, K, k, s, count in resnet50_convs(a.batch):
        x = torch.randn(N, C, H, W, device=dev, dtype=torch.bfloat16).to(memory_format=cl)
        w = (torch.randn(K, C, k, k, device=dev, dtype=torch.bfloat16) * 0.05).to(memory_format=cl)
        p = k // 2
        y = F.conv2d(x, w, stride=s, padding=p)
        dy = torch.randn_like(y)
        OH, OW = y.shape[2], y.shape[3]
        flops = 2.0 * N * OH * OW * K * C * k * k
        r = {"name": name, "N": N, "Cin": C, "H": H, "W": W, "Cout": K, "k": k, "stride": s,
             "count": count, "gflop": round(flops / 1e9, 2)}
        cb = torch.ops.aten.convolution_backward
        r["miopen_fwd_ms"] = timeit(lambda: F.conv2d(x, w, stride=s, padding=p), a.reps)
        r["miopen_dgrad_ms"] = timeit(lambda: cb(dy, x, w, None, [s, s], [p, p], [1, 1], False,
                                                 [0, 0], 1, [True, False, False]), a.reps)
        r["miopen_wgrad_ms"] = timeit(lambda: cb(dy, x, w, None, [s, s], [p, p], [1, 1], False,
                                                 [0, 0], 1, [False, True, False]), a.reps)
        mi = r["miopen_fwd_ms"] + r["miopen_dgrad_ms"] + r["miopen_wgrad_ms"]
        best = mi
        if k == 1 and s == 1:
            M = N * H * W
            X2 = x.permute(0, 2, 3, 1).reshape(M, C)
            W2 = w.reshape(K, C)
            D2 = dy.permute(0, 2, 3, 1).reshape(M, K)
            r["mm_fwd_ms"] = timeit(lambda: torch.mm(X2, W2.t()), a.reps)
            r["mm_dgrad_ms"] = timeit(lambda: torch.mm(D2, W2), a.reps)
            r["mm_wgrad_ms"] = timeit(lambda: torch.mm(D2.t(), X2), a.reps)
            S = 32 if M % 32 == 0 else 1
            Xs, Ds = X2.view(S, M // S, C), D2.view(S, M // S, K)
            r["bmm_splitk_wgrad_ms"] = timeit(
                lambda: torch.bmm(Ds.transpose(1, 2), Xs).float().sum(0), a.reps)
            best = (min(r["miopen_fwd_ms"], r["mm_fwd_ms"]) + min(r["miopen_dgrad_ms"], r["mm_dgrad_ms"])
                    + min(r["miopen_wgrad_ms"], r["mm_wgrad_ms"], r["bmm_splitk_wgrad_ms"]))
        for key in list(r):
            if key.endswith("_ms"):
                r[key] = round(r[key], 4)
                r[key.replace("_ms", "_tflops")] = round(flops / (r[key] * 1e-3) / 1e12, 1)
        total["miopen"] += mi * count
        total["best"] += best * count
        line = json.dumps(r)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "a") as fh:
                fh.write(line + "\n")
        del x, w, y, dy
        torch.cuda.empty_cache()
    print(json.dumps({"total_miopen_ms": round(total["miopen"], 3),
                      "total_best_ms": round(total["best"], 3)}), flush=True)


if __name__ == "__main__":
    main()
