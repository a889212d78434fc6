#!/usr/bin/env python3
"""Layer-1 3x3 conv kernels in isolation at the ResNet-50 batch-2048 shape (x [2048, 64, 56, 56]
NHWC bf16): the patch-resident kernel (conv3x3p.hip; forward, forward + BN statistics, data
gradient + BN-backward sums) with MFMA FLOP rates, through the same launchers the model calls.
CML_CONV3P_DBG (1 skip the MFMAs, 2 skip the per-tile patch DMA) times the kernel's skeleton.

  python bench/conv3x3p.py [--batch 2048] [--reps 20] [--json-out F]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps):
    fn()
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    from consensusml_amd.ops.native import lib
    L = lib()
    dev = torch.device("cuda")
    g0 = torch.Generator(device=dev).manual_seed(0)
    nh = lambda t: t.contiguous(memory_format=torch.channels_last)   # noqa: E731
    B = a.batch
    x = nh(torch.randn(B, 64, 56, 56, device=dev, generator=g0).bfloat16())
    z = nh(torch.randn(B, 64, 56, 56, device=dev, generator=g0).bfloat16())
    w = (torch.randn(64, 576, device=dev, generator=g0) * 0.04).bfloat16()
    zero = torch.zeros(64, device=dev, dtype=torch.bfloat16)
    sc = torch.rand(64, device=dev) + 0.5
    bi = torch.randn(64, device=dev) * 0.1
    mean, invstd = torch.zeros(64, device=dev), torch.ones(64, device=dev)
    fl = 2.0 * B * 56 * 56 * 64 * 576
    by = 2.0 * x.numel() * 2
    for name, fn in [("fwd", lambda: L.conv_gemm(x, w, 9, zero)),
                     ("fwd_stats", lambda: L.conv_gemm_bn(x, w, 9, zero)),
                     ("dgrad_bnsums", lambda: L.conv_gemm_bnsums(x, w, 9, zero, z, sc, bi, mean,
                                                                  invstd))]:
        ms = timeit(fn, a.reps)
        r = {"kernel": name, "batch": B, "dbg": os.environ.get("CML_CONV3P_DBG", "0"),
             "conv3p": os.environ.get("CML_CONV3P", "1"), "ms": round(ms, 4),
             "tflops": round(fl / ms / 1e9, 1), "io_TBps": round(by / ms / 1e9, 2)}
        print(json.dumps(r), flush=True)
        if a.json_out:
            with open(a.json_out, "a") as fh:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
