#!/usr/bin/env python3
"""Where does the fused 1x1 GEMM time go? Times conv1x1.hip (mode 0), the 2-buffer glds kernel
(mode 1) and the quad-phase kernel (mode 3) at a few compute-bound ResNet-50 shapes (batch 2048),
and the quad kernel with parts switched off (ablation bits, C1Args::ablate): 1 no MFMA, 2 no DMA,
4 no in-LDS prologue, 8 no epilogue (outputs are garbage then; timing only).

  python tools/diag/quad_ablate.py [--reps 10] [--only NAME] [--loop N]
  (--loop N: just run NAME's quad kernel N times, for rocprofv3 --pmc passes)
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = {   # name: (kind, batch, K1 (x channels), K2 (x2 channels), N, H)
    "l3.0_down_dx": ("cat", 2048, 1024, 512, 512, 14),
    "l4_conv1_dgrad": ("link", 2048, 512, 0, 2048, 7),
    "l4_conv3": ("bn_fwd_pro", 2048, 512, 0, 2048, 7),
    "l3.0_tail": ("cat_bnres", 2048, 256, 512, 1024, 14),
}


def timeit(fn, reps):
    for _ in range(3):
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


def build(name, dev):
    from consensusml_amd.ops.native import lib
    L = lib()
    kind, B, K1, K2, N, H = SHAPES[name]
    nh = lambda t: t.contiguous(memory_format=torch.channels_last)  # noqa: E731
    M = B * H * H
    g0 = torch.Generator(device=dev).manual_seed(0)
    if kind == "cat":
        g = nh(torch.randn(B, K1, H, H, device=dev, generator=g0).bfloat16())
        x2 = nh(torch.randn(B, K2, H, H, device=dev, generator=g0).bfloat16())
        mask = torch.randint(0, 256, (M, K1 // 8), device=dev, dtype=torch.uint8)
        bias = torch.randn(N, device=dev) * 0.1
        w = (torch.randn(N, K1 + K2, device=dev, generator=g0) * 0.03).bfloat16()
        # (a downsample data gradient: the block input x2 is staged as is)
        return lambda: L.conv1x1_cat(g, mask, x2, None, None, w, bias), 2.0 * M * (K1 + K2) * N
    if kind == "cat_bnres":
        x1 = nh(torch.randn(B, K1, H, H, device=dev, generator=g0).bfloat16())
        x2 = nh(torch.randn(B, K2, H, H, device=dev, generator=g0).bfloat16())
        sc = torch.rand(K1 + K2, device=dev) + 0.5
        bi = torch.randn(K1 + K2, device=dev) * 0.1
        w = (torch.randn(N, K1 + K2, device=dev, generator=g0) * 0.03).bfloat16()
        es, eb = torch.rand(N, device=dev) + 0.5, torch.randn(N, device=dev) * 0.1
        return (lambda: L.conv1x1_cat_bnres(x1, x2, sc[:K1], bi[:K1], None, None, w, es, eb),
                2.0 * M * (K1 + K2) * N)
    if kind == "link":
        x = nh(torch.randn(B, K1, H, H, device=dev, generator=g0).bfloat16())
        w = (torch.randn(N, K1, device=dev, generator=g0) * 0.03).bfloat16()
        link = nh(torch.randn(B, N, H, H, device=dev, generator=g0).bfloat16())
        lm = torch.randint(0, 256, (M, N // 8), device=dev, dtype=torch.uint8)
        return lambda: L.conv1x1_link(x, w, link, lm), 2.0 * M * K1 * N
    x = nh(torch.randn(B, K1, H, H, device=dev, generator=g0).bfloat16())
    w = (torch.randn(N, K1, 1, 1, device=dev, generator=g0) * 0.03).bfloat16()
    sc, bi = torch.rand(K1, device=dev) + 0.5, torch.randn(K1, device=dev) * 0.1
    rm, rv = torch.zeros(N, device=dev), torch.ones(N, device=dev)
    return (lambda: L.conv1x1_bn_fwd(x, w, sc, bi, rm, rm, rv, 1, True, 1e-5, 0.1),
            2.0 * M * K1 * N)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default=None)
    ap.add_argument("--loop", type=int, default=0)
    ap.add_argument("--mode", type=int, default=3)
    a = ap.parse_args()
    from consensusml_amd.ops.native import lib
    L = lib()
    dev = torch.device("cuda", 0)
    names = [a.only] if a.only else list(SHAPES)
    if a.loop:
        fn, _ = build(names[0], dev)
        L.set_conv1x1g_mode(a.mode)
        for _ in range(a.loop):
            fn()
        torch.cuda.synchronize()
        return
    for name in names:
        fn, fl = build(name, dev)
        r = {"name": name, "kind": SHAPES[name][0]}
        for label, mode, ab in (("old", 0, 0), ("glds2", 1, 0), ("quad", 3, 0),
                                ("quad_noMFMA", 3, 1), ("quad_noDMA", 3, 2),
                                ("quad_noPro", 3, 4), ("quad_noEpi", 3, 8),
                                ("quad_DMA_only", 3, 1 | 4 | 8), ("quad_MFMA_only", 3, 2 | 4 | 8),
                                ("quad_sync_only", 3, 1 | 2 | 4 | 8)):
            L.set_conv1x1g_mode(mode)
            L.set_conv1x1g_ablate(ab)
            t = timeit(fn, a.reps)
            r[label + "_ms"] = round(t, 4)
            r[label + "_tflops"] = round(fl / t / 1e9, 1)
        L.set_conv1x1g_ablate(0)
        L.set_conv1x1g_mode(2)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
