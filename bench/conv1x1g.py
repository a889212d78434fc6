#!/usr/bin/env python3
"""Per-shape A/B of the two fused 1x1-conv kernel families at the ResNet-50 step's shapes (batch
2048): conv1x1.hip (register-staged, persistent; ``set_conv1x1g_mode(0)``) vs conv1x1g.hip
(global_load_lds, 256-wide tiles; mode 1), through the same launchers the model calls, plus
hipBLASLt's plain GEMM of the same size as a reference point. Modes are interleaved per rep
(same process, same data).

  python bench/conv1x1g.py [--batch 2048] [--reps 10] [--json-out F]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (launcher, name, H, K1, K2 / K, N): every fused 1x1 launch of the step with N % 128 == 0
CASES = [
    ("bn_fwd", "l2.0_conv1", 56, 256, 0, 128), ("bn_fwd", "l2_conv1", 28, 512, 0, 128),
    ("bn_fwd", "l3.0_conv1", 28, 512, 0, 256),
    ("bn_fwd_pro", "l4_conv3", 7, 512, 0, 2048),
    ("link", "l2_conv1_dgrad", 28, 128, 0, 512), ("link", "l3_conv1_dgrad", 14, 256, 0, 1024),
    ("link", "l4_conv1_dgrad", 7, 512, 0, 2048),
    ("link_sums", "l3_conv1_dgrad_sums", 14, 256, 0, 1024),
    ("link_s2", "l2.0_conv1_dgrad", 56, 128, 0, 256), ("link_s2", "l3.0_conv1_dgrad", 28, 256, 0, 512),
    ("bnres", "l2_tail", 28, 128, 0, 512), ("bnres", "l3_tail", 14, 256, 0, 1024),
    ("cat", "l2_tail_dgrad", 28, 512, 128, 128), ("cat", "l3_tail_dgrad", 14, 1024, 256, 256),
    ("cat", "l2.0_down_dx", 28, 512, 256, 256), ("cat", "l3.0_down_dx", 14, 1024, 512, 512),
    ("cat_bnsums", "l2_tail_dgrad_sums", 28, 512, 128, 128),
    ("cat_bnsums", "l3_tail_dgrad_sums", 14, 1024, 256, 256),
    ("cat_bnres", "l2.0_tail", 28, 128, 256, 512), ("cat_bnres", "l3.0_tail", 14, 256, 512, 1024),
]


def timeit(fns, reps):
    """Median ms of each fn, interleaved per rep."""
    for f in fns:
        f()
        f()
    ts = [[] for _ in fns]
    for _ in range(reps):
        for i, f in enumerate(fns):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            f()
            b.record()
            b.synchronize()
            ts[i].append(a.elapsed_time(b))
    return [sorted(t)[len(t) // 2] for t in ts]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default=None)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    from consensusml_amd.ops.native import lib
    L = lib()
    dev = torch.device("cuda")
    B = a.batch
    g0 = torch.Generator(device=dev).manual_seed(0)
    nh = lambda t: t.contiguous(memory_format=torch.channels_last)   # noqa: E731
    tot = {"old": 0.0, "quad": 0.0}
    for kind, name, H, K1, K2, N in CASES:
        if a.only and a.only not in name:
            continue
        K = K1 + K2
        M = B * H * H
        x = nh(torch.randn(B, K1, H, H, device=dev, generator=g0).bfloat16())
        if kind in ("bn_fwd", "bn_fwd_pro"):
            w = (torch.randn(N, K, 1, 1, device=dev, generator=g0) * K ** -0.5).bfloat16()
            sc = torch.rand(K, device=dev) + 0.5 if kind == "bn_fwd_pro" else None
            bi = torch.randn(K, device=dev) * 0.1 if kind == "bn_fwd_pro" else None
            rm, rv = torch.zeros(N, device=dev), torch.ones(N, device=dev)
            fn = lambda: L.conv1x1_bn_fwd(x, w, sc, bi, rm, rm, rv, 1, True, 1e-5, 0.1)  # noqa
        elif kind in ("link", "link_sums"):
            w = (torch.randn(N, K, device=dev, generator=g0) * K ** -0.5).bfloat16()
            link = nh(torch.randn(B, N, H, H, device=dev, generator=g0).bfloat16())
            lm = torch.randint(0, 256, (M, N // 8), device=dev, dtype=torch.uint8)
            extra = ()
            if kind == "link_sums":
                extra = (nh(torch.randn(B, N, H, H, device=dev).bfloat16()),
                         torch.randint(0, 256, (M, N // 8), device=dev, dtype=torch.uint8),
                         torch.zeros(N, device=dev), torch.ones(N, device=dev))
            fn = lambda: L.conv1x1_link(x, w, link, lm, *extra)  # noqa: E731
        elif kind == "link_s2":
            # x: the stride-1 gradient dy [B, K, H, H] of conv1; link: the compact downsample
            # gradient [B, N, H/2, H/2]
            w = (torch.randn(N, K, device=dev, generator=g0) * K ** -0.5).bfloat16()
            g = nh(torch.randn(B, N, (H + 1) // 2, (H + 1) // 2, device=dev).bfloat16())
            fn = lambda: L.conv1x1_link_s2(x, w, g)  # noqa: E731
        elif kind == "bnres":
            w = (torch.randn(N, K, 1, 1, device=dev, generator=g0) * K ** -0.5).bfloat16()
            sc, bi = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.1
            s3, b3 = torch.rand(N, device=dev) + 0.5, torch.randn(N, device=dev) * 0.1
            res = nh(torch.randn(B, N, H, H, device=dev).bfloat16())
            fn = lambda: L.conv1x1_bnres(x, w, sc, bi, s3, b3, res)  # noqa: E731
        else:
            x2 = nh(torch.randn(B, K2, H, H, device=dev, generator=g0).bfloat16())
            w = (torch.randn(N, K, device=dev, generator=g0) * K ** -0.5).bfloat16()
            sc, bi = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.1
            # as the model calls them: the downsample GEMMs stage the block input x2 as is
            sc2, bi2 = (None, None) if kind == "cat_bnres" or "down" in name else (sc[K1:], bi[K1:])
            if kind == "cat_bnres":
                es, eb = torch.rand(N, device=dev) + 0.5, torch.randn(N, device=dev) * 0.1
                fn = lambda: L.conv1x1_cat_bnres(x, x2, sc[:K1], bi[:K1], sc2, bi2, w, es, eb)  # noqa
            else:
                mask = torch.randint(0, 256, (M, K1 // 8), device=dev, dtype=torch.uint8)
                bias = torch.randn(N, device=dev) * 0.1
                if kind == "cat":
                    fn = lambda: L.conv1x1_cat(x, mask, x2, sc2, bi2, w, bias)  # noqa: E731
                else:
                    mu, iv = torch.zeros(N, device=dev), torch.ones(N, device=dev)
                    fn = lambda: L.conv1x1_cat_bnsums(x, mask, x2, sc2, bi2, w, bias, mu, iv)  # noqa

        def in_mode(m):
            def f():
                L.set_conv1x1g_mode(m)
                fn()
            return f
        xa = torch.randn(M, K, device=dev).bfloat16()
        wa = torch.randn(K, N, device=dev).bfloat16()
        t_old, t_q, t_mm = timeit([in_mode(0), in_mode(3), lambda: torch.mm(xa, wa)], a.reps)
        L.set_conv1x1g_mode(2)
        fl = 2.0 * M * K * N
        r = {"kind": kind, "name": name, "M": M, "K": K, "N": N, "old_ms": round(t_old, 4),
             "quad_ms": round(t_q, 4),
             "speedup_quad": round(t_old / t_q, 3),
             "old_tflops": round(fl / t_old / 1e9, 1),
             "quad_tflops": round(fl / t_q / 1e9, 1),
             "hipblaslt_mm_ms": round(t_mm, 4), "hipblaslt_tflops": round(fl / t_mm / 1e9, 1)}
        tot["old"] += t_old
        tot["quad"] += t_q
        print(json.dumps(r), flush=True)
        if a.json_out:
            with open(a.json_out, "a") as fh:
                fh.write(json.dumps(r) + "\n")
        del x, xa, wa
        torch.cuda.empty_cache()
    print(json.dumps({"total_ms": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
