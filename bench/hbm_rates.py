#!/usr/bin/env python3
"""HBM stream rates on one MI355X for the access mixes the memory-bound kernels have: read-only
(sum), write-only (fill / zero), copy (1 read : 1 write) and add (2 : 1). One JSON line per case;
TB/s counts read + write bytes. 2 GiB operands (beyond the 256 MB last-level cache).

  python bench/hbm_rates.py
"""
import json
import os

import torch


def _t(fn, it=10):
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
    dev = torch.device("cuda")
    n = int(os.environ.get("HBM_N", 1 << 30))   # 1 G bf16 elements = 2 GiB
    a = torch.randn(n, device=dev, dtype=torch.bfloat16)
    b = torch.randn(n, device=dev, dtype=torch.bfloat16)
    c = torch.empty(n, device=dev, dtype=torch.bfloat16)
    s = torch.empty((), device=dev, dtype=torch.float32)
    cases = [
        ("read_sum", lambda: torch.sum(a, 0, dtype=torch.float32, out=s), 2 * n),
        ("write_fill", lambda: c.fill_(1.0), 2 * n),
        ("write_zero", lambda: c.zero_(), 2 * n),
        ("copy", lambda: c.copy_(a), 4 * n),
        ("add_2r1w", lambda: torch.add(a, b, out=c), 6 * n),
    ]
    for name, fn, byt in cases:
        t = _t(fn)
        print(json.dumps({"case": name, "gb": round(byt / 1e9, 2), "us": round(t * 1e6, 1),
                          "tb_s": round(byt / t / 1e12, 2)}), flush=True)


if __name__ == "__main__":
    main()
