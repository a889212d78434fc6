#!/usr/bin/env python3
"""The ResNet-50 1x1-conv GEMMs that ``ops.conv.conv_mm`` runs on gemm.hip at batch 2048 (layers
3-4: forwards with cin >= 1024 and data gradients, some with the parked residual gradient added in
the epilogue), on the 256 x 256 kernel (the model's choice) vs the 128 x 128 kernel
(gemm128.hip, 4x the tiles: a smaller last wave on 256 CUs) vs hipBLASLt. One JSON line per shape.

  python bench/conv_mm_tiles.py [--batch B]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(it):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2] * 1e-3


def main():
    from consensusml_amd.ops.native import lib
    L = lib()
    B = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 2048
    dev = torch.device("cuda")
    m3, m4 = B * 14 * 14, B * 7 * 7
    # (name, M, K, N, residual acc)
    shapes = [("l3_fwd_1024_256", m3, 1024, 256, False), ("l3_dgrad_c3_1024_256", m3, 1024, 256, True),
              ("l3_dgrad_c1_256_1024", m3, 256, 1024, True), ("l4_fwd_2048_512", m4, 2048, 512, False),
              ("l4_dgrad_c3_2048_512", m4, 2048, 512, True), ("l4_dgrad_c1_512_2048", m4, 512, 2048, True)]
    g = torch.Generator(device=dev).manual_seed(0)
    for name, M, K, N, res in shapes:
        a = torch.randn(M, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).bfloat16()
        acc = torch.randn(M, N, device=dev, generator=g).bfloat16() if res else None
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        row = {"case": name, "M": M, "K": K, "N": N, "acc": res}
        ref = None
        for tile in (256, 128):
            ok = (L.gemm_nt_ok(M, N, K) if tile == 256 else
                  (M % 128 == 0 and N % 128 == 0 and K % 64 == 0))
            if not ok:
                continue
            if res:
                fn = lambda t=tile: L.gemm_nt(a, w, 0, out=out, cin=acc, tile=t)
            else:
                fn = lambda t=tile: L.gemm_nt(a, w, 0, out=out, tile=t)
            fn()
            y = out.float()
            if ref is None:
                ref = y.clone()
            row[f"t{tile}_us"] = round(_t(fn) * 1e6, 1)
            row[f"t{tile}_tflops"] = round(2.0 * M * N * K / (row[f"t{tile}_us"] * 1e-6) / 1e12, 1)
            row[f"t{tile}_maxdiff_vs_t256"] = float((y - ref).abs().max())
        fb = (lambda: torch.addmm(acc, a, w.t())) if res else (lambda: torch.mm(a, w.t()))
        row["hipblaslt_us"] = round(_t(fb) * 1e6, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
