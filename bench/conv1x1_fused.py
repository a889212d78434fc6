#!/usr/bin/env python3
"""Per-shape timing of the fused 1x1 conv + BN statistics kernel (csrc/kernels/conv1x1.hip)
against what it replaces in the ResNet-50 step: the library conv (MIOpen, or hipBLASLt where
``models.resnet.conv1x1_policy`` picks a GEMM) plus the BN statistics pass (``bn_stats``), and
for conv3 also bn2's apply pass (its output y2 is what the library conv reads).

  python bench/conv1x1_fused.py --batch 2048 [--json-out gpurun_out/conv1x1.jsonl]

One JSON line per shape: ms of each variant (median of --reps after warmup, CUDA events), and the
fused kernel's achieved HBM rate (x read once, y written once).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (name, Cin, Cout, H_in, stride, prologue) of every 1x1 conv of ResNet-50 (one per distinct shape)
SHAPES = [
    ("l1_conv1_b0", 64, 64, 56, 1, False), ("l1_conv1", 256, 64, 56, 1, False),
    ("l1_conv3", 64, 256, 56, 1, True), ("l1_down", 64, 256, 56, 1, False),
    ("l2_conv1_b0", 256, 128, 56, 1, False), ("l2_conv1", 512, 128, 28, 1, False),
    ("l2_conv3", 128, 512, 28, 1, True), ("l2_down", 256, 512, 56, 2, False),
    ("l3_conv1_b0", 512, 256, 28, 1, False), ("l3_conv1", 1024, 256, 14, 1, False),
    ("l3_conv3", 256, 1024, 14, 1, True), ("l3_down", 512, 1024, 28, 2, False),
    ("l4_conv1_b0", 1024, 512, 14, 1, False), ("l4_conv1", 2048, 512, 7, 1, False),
    ("l4_conv3", 512, 2048, 7, 1, True), ("l4_down", 1024, 2048, 14, 2, False),
]


def timeit(fn, reps: int, warm: int = 3) -> float:
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default=None)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    from consensusml_amd.ops.native import lib
    from consensusml_amd.models.resnet import conv1x1_policy
    from consensusml_amd.utils.tuning import configure_miopen
    configure_miopen()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    L = lib()
    out = []
    for name, ci, co, H, st, pro in SHAPES:
        if a.only and a.only not in name:
            continue
        B = a.batch
        x = torch.randn(B, ci, H, H, device=dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = (torch.randn(co, ci, 1, 1, device=dev) / ci ** 0.5).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        rm = torch.zeros(co, device=dev)
        rv = torch.ones(co, device=dev)
        sc = torch.rand(ci, device=dev) + 0.5
        bi = torch.randn(ci, device=dev) * 0.1
        g = torch.ones(ci, device=dev, dtype=torch.bfloat16)
        be = torch.zeros(ci, device=dev, dtype=torch.bfloat16)
        mi = torch.zeros(ci, device=dev)
        iv = torch.ones(ci, device=dev)
        OH = H // st
        fwd_gemm = st == 1 and conv1x1_policy(ci, co, H * H)[0]

        def lib_conv(inp):
            if fwd_gemm:
                return torch.mm(inp.permute(0, 2, 3, 1).reshape(-1, ci), w.view(co, ci).t())
            return F.conv2d(inp, w, stride=st)

        def base():
            inp = x
            if pro:   # bn2 apply pass writes y2, which the library conv reads
                inp = L.bn_fwd(x, None, g, be, None, None, mi, iv, 1e-5, 0.1, True, False,
                               False)[0]
            y = lib_conv(inp)
            if y.dim() == 2:
                y = y.view(B, OH, OH, co).permute(0, 3, 1, 2)
            L.bn_stats(y, rm, rv, 1e-5, 0.1)

        def fused():
            L.conv1x1_bn_fwd(x, w, sc if pro else None, bi if pro else None, rm, rm, rv, st,
                             True, 1e-5, 0.1)

        tb = timeit(base, a.reps)
        tf = timeit(fused, a.reps)
        tl = timeit(lambda: lib_conv(x), a.reps)
        gb = (x.numel() * 2 / (st * st) + B * OH * OH * co * 2) / 1e9
        flop = 2.0 * B * OH * OH * ci * co
        r = {"name": name, "batch": B, "cin": ci, "cout": co, "h": H, "stride": st, "prologue": pro,
             "library": "hipblaslt" if fwd_gemm else "miopen", "library_conv_ms": round(tl, 4),
             "unfused_ms": round(tb, 4), "fused_ms": round(tf, 4),
             "saved_ms": round(tb - tf, 4), "fused_tb_s": round(gb / tf, 2),
             "fused_tflops": round(flop / tf / 1e9, 1)}
        out.append(r)
        print(json.dumps(r), flush=True)
        if a.json_out:
            with open(a.json_out, "a") as fh:
                fh.write(json.dumps(r) + "\n")
        del x, w
        torch.cuda.empty_cache()
    tot = {k: round(sum(r[k] for r in out), 3) for k in ("unfused_ms", "fused_ms", "saved_ms")}
    print(json.dumps({"total": tot}), flush=True)


if __name__ == "__main__":
    main()
