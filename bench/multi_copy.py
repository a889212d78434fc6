"""Gradient-capture copy (csrc/kernels/multi_copy.hip) throughput on two entry mixes: the
parameter tensors of a ResNet-50 bucket (hundreds of small tensors) and Llama-3-8B-sized weight
gradients (four 34-117 MB tensors). Emits one JSON line per case; TB/s counts read + write.

    python bench/multi_copy.py [--reps R]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from consensusml_amd.ops.native import lib  # noqa: E402


def _case(name, sizes, reps, dev):
    src = [torch.randn(s, device=dev, dtype=torch.bfloat16) for s in sizes]
    buf = torch.empty(sum((s + 63) // 64 * 64 for s in sizes), device=dev, dtype=torch.bfloat16)
    dst, off = [], 0
    for s in sizes:
        dst.append(buf[off:off + s])
        off += (s + 63) // 64 * 64
    for _ in range(3):
        assert not lib().multi_copy(dst, src)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(0, len(dst), 32):
            lib().multi_copy(dst[i:i + 32], src[i:i + 32])
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    t = sorted(ts)[len(ts) // 2] * 1e-3
    byt = 2 * 2 * sum(sizes)
    ok = all(torch.equal(d, s) for d, s in zip(dst, src))
    print(json.dumps({"case": name, "entries": len(sizes), "mb": round(byt / 2 / 1e6, 1),
                      "us": round(t * 1e6, 1), "tb_s": round(byt / t / 1e12, 2), "exact": ok}),
          flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda")
    from consensusml_amd.models.resnet import resnet50
    m = resnet50()
    sizes = [p.numel() for p in m.parameters()]
    # one ~8 MB bucket's worth of consecutive parameters, and the whole model
    acc, bucket = 0, []
    for s in sizes[::-1]:
        bucket.append(s)
        acc += 2 * s
        if acc >= 8 << 20:
            break
    _case("resnet50_bucket_8mb", bucket, args.reps, dev)
    _case("resnet50_all", sizes, args.reps, dev)
    _case("llama8b_layer_weights", [4096 * 6144, 4096 * 4096, 2 * 14336 * 4096, 4096 * 14336],
          args.reps, dev)
    # speed of light: one contiguous device copy of the same bytes (ATen / the runtime's blit)
    n = 4096 * 6144 + 4096 * 4096 + 3 * 14336 * 4096
    a, b = (torch.empty(n, device=dev, dtype=torch.bfloat16) for _ in range(2))
    for _ in range(3):
        b.copy_(a)
    torch.cuda.synchronize()
    ts = []
    for _ in range(args.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.copy_(a)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    t = sorted(ts)[len(ts) // 2] * 1e-3
    print(json.dumps({"case": "aten_copy_same_bytes", "mb": round(2 * n / 1e6, 1),
                      "us": round(t * 1e6, 1), "tb_s": round(4 * n / t / 1e12, 2)}), flush=True)


if __name__ == "__main__":
    main()
