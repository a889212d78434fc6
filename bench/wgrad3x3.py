#!/usr/bin/env python3
"""3x3 stride-1 weight gradients of ResNet-50 at batch 2048: MIOpen (aten convolution_backward,
channels_last bf16) vs csrc/kernels/wgrad3x3.hip (nine taps per workgroup) (the one-tap-per-grid-z variant was removed in round 3)
TAP mode of wgrad1x1.hip. One JSON line per shape (ms, PFLOP/s, relative error vs fp32 on a slice).

  python bench/wgrad3x3.py [--json-out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _t(fn, it=10):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--json-out", default=None)
    args = ap.parse_args()
    from consensusml_amd.ops.native import lib
    from consensusml_amd.utils.tuning import configure_miopen
    configure_miopen()
    torch.backends.cudnn.benchmark = True
    L = lib()
    dev = torch.device("cuda:0")
    zero = torch.zeros(64, dtype=torch.bfloat16, device=dev)
    rows = []
    for C, H in ((64, 56), (128, 28), (256, 14), (512, 7)):
        B = args.batch
        x = torch.randn(B, C, H, H, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        gy = torch.randn(B, C, H, H, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = torch.zeros(C, C, 3, 3, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        flops = 2 * B * H * H * 9 * C * C
        t_lib = _t(lambda: torch.ops.aten.convolution_backward(
            gy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))
        t_dir = _t(lambda: L.wgrad3x3(gy, x, torch.bfloat16, zero))
        xs, gs = x[:16].contiguous(memory_format=torch.channels_last), \
            gy[:16].contiguous(memory_format=torch.channels_last)
        ref = torch.ops.aten.convolution_backward(gs.float(), xs.float(), w.float(), None, [1, 1],
                                                  [1, 1], [1, 1], False, [0, 0], 1,
                                                  [False, True, False])[1]
        d = L.wgrad3x3(gs, xs, torch.float32, zero)
        err = float((d.float() - ref).norm() / ref.norm())
        r = {"C": C, "H": H, "batch": B, "miopen_ms": round(t_lib, 4), "direct_ms": round(t_dir, 4),
             "miopen_pflops": round(flops / t_lib / 1e12, 3),
             "direct_pflops": round(flops / t_dir / 1e12, 3),
             "direct_ok": bool(L.wgrad3x3_direct_ok(B, H, H, C, C)), "direct_rel_err": err}
        print(json.dumps(r), flush=True)
        rows.append(r)
        del x, gy
        torch.cuda.empty_cache()
    if args.json_out:
        with open(args.json_out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
