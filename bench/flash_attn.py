#!/usr/bin/env python3
"""Flash attention (csrc/kernels/flash_attn.hip) vs ROCm SDPA (AOTriton) at the Llama-3-8B shape.

One JSON line per (impl, pass): ms per call (median of --iters after warmup, HIP events) and
TFLOP/s of causal attention (forward 2 S^2 hd H B of useful work = 4 B H S^2 hd / 2; backward
2.5x the forward's products). Random data (zero-filled inputs collapse the softmax work).

  python bench/flash_attn.py --B 4 --S 2048
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--H", type=int, default=32)
    ap.add_argument("--KV", type=int, default=8)
    ap.add_argument("--S", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--full", action="store_true", help="non-causal")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--impl", default="flash,flash_thr0,sdpa")
    a = ap.parse_args()
    from consensusml_amd.ops.native import lib
    B, H, KV, S, D = a.B, a.H, a.KV, a.S, 128
    causal = not a.full
    scale = D ** -0.5
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(B, H, S, D, device="cuda", generator=g).bfloat16()
    k = torch.randn(B, KV, S, D, device="cuda", generator=g).bfloat16()
    v = torch.randn(B, KV, S, D, device="cuda", generator=g).bfloat16()
    do = torch.randn(B, S, H * D, device="cuda", generator=g).bfloat16()
    fwd_flop = 4.0 * B * H * S * S * D * (0.5 if causal else 1.0)
    L = lib()
    fns = {}
    for impl in a.impl.split(","):
        if impl in ("flash", "flash_thr0"):
            thr = 8.0 if impl == "flash" else 0.0    # deferred-rescale threshold (log2 units)
            o, lse = L.flash_fwd(q, k, v, causal, scale, thr)
            fns[impl] = (lambda thr=thr: L.flash_fwd(q, k, v, causal, scale, thr),
                         lambda o=o, lse=lse: L.flash_bwd(q, k, v, o, do, lse, causal, scale))
        else:
            qa, ka, va = (t.clone().requires_grad_() for t in (q, k, v))

            def run_f(qa=qa, ka=ka, va=va):
                return F.scaled_dot_product_attention(qa, ka, va, is_causal=causal, scale=scale,
                                                      enable_gqa=H != KV)
            out = run_f()
            dos = do.view(B, S, H, D).transpose(1, 2)
            fns[impl] = (run_f, lambda out=out, qa=qa, ka=ka, va=va: torch.autograd.grad(
                out, (qa, ka, va), dos, retain_graph=True))
    # interleaved rounds in one process (variants share the clock / thermal state)
    res = {(i, p): [] for i in fns for p in ("fwd", "bwd")}
    for _ in range(a.rounds):
        for impl, (fwd, bwd) in fns.items():
            for name, fn in (("fwd", fwd), ("bwd", bwd)):
                med, _ = timed(fn, a.iters, a.warmup)
                res[(impl, name)].append(med)
    for (impl, name), ts in res.items():
        ts.sort()
        flop = fwd_flop * (1.0 if name == "fwd" else 2.5)
        med = ts[len(ts) // 2]
        print(json.dumps({"bench": "flash_attn", "impl": impl, "pass": name, "B": B, "H": H,
                          "KV": KV, "S": S, "causal": causal, "ms": round(med, 4),
                          "ms_min": round(ts[0], 4), "rounds": a.rounds,
                          "tflops": round(flop / med / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
