#!/usr/bin/env python3
"""Driver for the rocprofv3 --pmc passes over this round's hot kernels (one process, a few
dispatches each, real shapes):

  agg     the consensus step at n = 8 virtual workers on D = 25.6 M bf16 coordinates (ResNet-50's
          size; synthetic worker gradients, no model compute): per-bucket Gram stage 1
          (gram_partial), the deferred multi-bucket reduce (gram_reduce_multi), the Krum weights
          (robust_weights) and the one-launch multi-bucket rule + SGD update (agg_update_multi:
          weighted combine for Krum, sorted for the median)
  flash   flash attention forward + backward, Llama-3-8B layer (B 4, 32 q / 8 kv heads, S 2048,
          hd 128, causal)
  gemm    gemm.hip (8 waves) and gemm_w4.hip (4 waves, modes 0 / 2 / 3) at 8192^3 and the Llama
          w13 shapes; gemm128.hip at the BERT per-rank fc2 shape (8192 x 768 x 3072)
  stem    the stem weight gradient with the pool-gradient gather (stem_wgrad_pool) at the bench
          shape (batch 2560, 224 x 224), parity-class staging on and off (CML_STEM_CLS)
  wgrad   the LDS-DMA 1x1 weight gradient (wgrad1x1.hip) at ResNet-50 layer-3 (1024 -> 256,
          batch 2048: 401 408 pixels) and a Llama projection (4096 x 4096 over 8192 tokens)

  rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d OUT -o run -- python3 tools/diag/pmc_targets.py
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def rnd(shape, dev, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    return (torch.rand(*shape, generator=g, device=dev) * 2 - 1).bfloat16()


def run_agg(dev, steps):
    """The engine's consensus step on synthetic worker gradients (no model compute): 8 virtual
    workers x D = 25.6 M bf16 coordinates (ResNet-50's size, one 64 MB bucket), sharded topology
    at one rank: per-bucket Gram stage 1, the deferred multi-bucket reduce, the weights launch and
    the one-launch multi-bucket rule + SGD update."""
    from consensusml_amd import TrainConfig
    from consensusml_amd.parallel.dist import DistInfo
    from consensusml_amd.parallel.engine import ConsensusEngine
    for rule in ("krum", "median"):
        cfg = TrainConfig()
        cfg.virtual_workers = 8
        cfg.agg.rule = rule
        cfg.agg.f = 2
        cfg.topology.kind = "sharded"
        model = torch.nn.Linear(5056, 5056, bias=False).to(dev).bfloat16()   # 25.56 M params
        eng = ConsensusEngine(model, cfg, DistInfo(0, 1, 0, dev, "none"))
        g = torch.Generator(device=dev).manual_seed(0)
        base = torch.randn(eng.flat.total, generator=g, device=dev)
        X = (base + 0.01 * torch.randn(8, eng.flat.total, generator=g, device=dev))
        for _ in range(steps):
            eng.zero_grad()
            eng.flat.flat_grad.copy_(X.to(eng.flat.flat_grad.dtype))
            eng._flushed = {b.index for b in eng.flat.buckets}
            eng.step()
            torch.cuda.synchronize()
            print("agg", rule, "step", flush=True)
        del eng, model, X, base
        torch.cuda.empty_cache()


def run_flash(dev, steps):
    from consensusml_amd.ops.transformer import flash_attention
    B, H, KV, S, D = 4, 32, 8, 2048, 128
    q = rnd((B, H, S, D), dev, 1).requires_grad_()
    k = rnd((B, KV, S, D), dev, 2).requires_grad_()
    v = rnd((B, KV, S, D), dev, 3).requires_grad_()
    do = rnd((B, S, H * D), dev, 4)
    for _ in range(steps):
        o = flash_attention(q, k, v, causal=True)
        o.backward(do)
    torch.cuda.synchronize()


def run_gemm(dev, steps):
    from consensusml_amd.ops.native import lib
    L = lib()
    n = 8192
    x, w = rnd((n, n), dev, 5), rnd((n, n), dev, 6)
    y = torch.empty(n, n, dtype=torch.bfloat16, device=dev)
    for _ in range(steps):
        L.gemm_nt(x, w, 0, out=y, tile=256)
        L.gemm_w4(x, w, 0, out=y)
    del x, w, y
    M, N, K = 8192, 28672, 4096       # Llama w13: forward, data gradient, weight gradient
    x, w, dy = rnd((M, K), dev, 7), rnd((N, K), dev, 8), rnd((M, N), dev, 9)
    for _ in range(steps):
        L.gemm_w4(x, w, 0)
        L.gemm_w4(dy, w, 2)
        L.gemm_w4(dy, x, 3)
    del x, w, dy
    a, b = rnd((8192, 3072), dev, 10), rnd((768, 3072), dev, 11)
    for _ in range(steps):
        L.gemm_nt(a, b, 0, tile=128)
    torch.cuda.synchronize()


def run_stem(dev, steps):
    from consensusml_amd.ops.native import lib
    from consensusml_amd.ops.stem import pack_stem_weight
    L = lib()
    N = 2560
    x = rnd((N, 224, 224, 3), dev, 14).permute(0, 3, 1, 2)   # channels-last [N, 3, 224, 224]
    w = (rnd((64, 3, 7, 7), dev, 15).float() * 0.1).bfloat16()
    gam = (rnd((64,), dev, 16).float() * 0.5 + 1).bfloat16()
    bet = (rnd((64,), dev, 17).float() * 0.2).bfloat16()
    z, mean, invstd = L.stem_conv_fwd(x, pack_stem_weight(w), None, None, 1e-5, 0.1, True)
    y, idx, _, _ = L.bn_relu_maxpool_fwd(z, gam, bet, None, None, mean, invstd, 1e-5, 0.1,
                                         False, 3, 2, 1)
    dy = rnd(tuple(y.shape), dev, 18).view(y.shape[0], y.shape[2], y.shape[3], y.shape[1]) \
        .permute(0, 3, 1, 2)
    for cls in ("1", "0"):
        os.environ["CML_STEM_CLS"] = cls
        for _ in range(steps):
            L.stem_wgrad_pool(dy, idx, None, z, x, mean, invstd, gam)
        torch.cuda.synchronize()
        print("stem cls", cls, flush=True)
    os.environ.pop("CML_STEM_CLS", None)


def run_wgrad(dev, steps):
    from consensusml_amd.ops.native import lib
    L = lib()

    def nhwc(t2):
        T, C = t2.shape
        return t2.view(T, 1, 1, C).permute(0, 3, 1, 2)
    for T, Cin, Cout in ((2048 * 14 * 14, 1024, 256), (8192, 4096, 4096)):
        x, dy = rnd((T, Cin), dev, 12), rnd((T, Cout), dev, 13)
        for _ in range(steps):
            L.wgrad1x1(nhwc(dy), nhwc(x), torch.bfloat16)
        del x, dy
    torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=["agg", "flash", "gemm", "wgrad"])
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for name in a.only:
        globals()["run_" + name](dev, a.steps)
        print("done", name, flush=True)


if __name__ == "__main__":
    main()
