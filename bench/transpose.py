#!/usr/bin/env python3
"""bf16 transpose (``transpose_bf16``: the operand transposes of the NT weight gradients and the
weight transposes of the data gradients) at the Llama-3-8B shapes vs ATen's ``t().contiguous()``.
TB/s counts read + write; the operand stays cache-warm across the timed repeats (64-470 MB), so
these are upper bounds for the in-step calls. One JSON line per shape. (A register-only 8 x 8
transpose kernel measured the same here and in the Llama step, profiles/r05_46/.)

  python bench/transpose.py
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
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e-3


def main():
    from consensusml_amd.ops.native import lib
    L = lib()
    dev = torch.device("cuda")
    for R, C in ((8192, 4096), (8192, 14336), (8192, 28672), (4096, 14336), (6144, 4096)):
        x = torch.randn(R, C, device=dev).bfloat16()
        y = L.transpose_bf16(x)
        ok = torch.equal(y, x.t().contiguous())
        t = _t(lambda: L.transpose_bf16(x))
        ta = _t(lambda: x.t().contiguous())
        byt = 4 * R * C
        print(json.dumps({"R": R, "C": C, "us": round(t * 1e6, 1),
                          "tb_s": round(byt / t / 1e12, 2), "aten_us": round(ta * 1e6, 1),
                          "exact": ok}), flush=True)


if __name__ == "__main__":
    main()
