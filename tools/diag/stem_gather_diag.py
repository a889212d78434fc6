#!/usr/bin/env python3
"""Stem backward: gather path (stem_wgrad_pool) vs two-pass path (maxpool_bwd_sum + stem_wgrad)
over batch sizes, and vs float64 where it fits; per-output differences (dW, dgamma, dbeta)."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def main():
    from consensusml_amd.ops.native import lib
    from consensusml_amd.ops.stem import pack_stem_weight
    L = lib()
    dev = torch.device("cuda:0")
    for N in [2, 8, 32, 128, 512, 2048]:
        torch.manual_seed(0)
        x = torch.randn(N, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = (torch.randn(64, 3, 7, 7, device=dev) * 0.1).to(torch.bfloat16)
        gam = torch.empty(64, device=dev).uniform_(0.5, 1.5).to(torch.bfloat16)
        bet = torch.empty(64, device=dev).uniform_(-0.2, 0.2).to(torch.bfloat16)
        z, mean, invstd = L.stem_conv_fwd(x, pack_stem_weight(w), None, None, 1e-5, 0.1, True)
        y, idx, _, _ = L.bn_relu_maxpool_fwd(z, gam, bet, None, None, mean, invstd, 1e-5, 0.1,
                                             False, 3, 2, 1)
        dy = torch.randn_like(y)
        dw, dg, db = L.stem_wgrad_pool(dy, idx, None, z, x, mean, invstd, gam)
        g, gsum = L.maxpool_bwd_sum(dy, idx, z.shape[2], z.shape[3], None)
        dw2, dg2, db2 = L.stem_wgrad(g, z, x, mean, invstd, gam, gsum)
        r = {"N": N, "dw": rel(dw, dw2), "dg": rel(dg, dg2), "db": rel(db, db2),
             "gsum_vs_g": rel(gsum, g.float().sum((0, 2, 3)))}
        if N <= 32:
            gd = g.double()
            xh = (z.double() - mean.double().view(1, -1, 1, 1)) * invstd.double().view(1, -1, 1, 1)
            s1, s2 = gd.sum((0, 2, 3)), (gd * xh).sum((0, 2, 3))
            M = gd.numel() / 64
            sc = (gam.double() * invstd.double()).view(1, -1, 1, 1)
            dz = sc * (gd - s1.view(1, -1, 1, 1) / M - xh * (s2.view(1, -1, 1, 1) / M))
            wq = w.double().requires_grad_(True)
            F.conv2d(x.double(), wq, stride=2, padding=3).backward(dz)
            r["dw_gather_vs_f64"] = rel(dw, wq.grad)
            r["dw_two_vs_f64"] = rel(dw2, wq.grad)
            del gd, xh, dz, wq
        print(json.dumps(r), flush=True)
        del x, z, y, idx, dy, g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
