#!/usr/bin/env python3
"""HBM stream-rate probes (tools/diag/hbm_copy.hip, loaded with ctypes): copy (1 read : 1 write),
add (2 : 1) and fill, with 1-8 16-B vectors in flight per thread, one-pass or grid-stride grids
of 1-8 workgroups per CU, plain or nontemporal loads / stores, interleaved in one process against
PyTorch's copy_ / add / fill_. 2 GiB operands (beyond the 256 MB last-level cache). TB/s counts
read + write bytes. One JSON line per case.

  python tools/diag/hbm_copy.py [--so build/hbm_copy.so]
"""
import argparse
import ctypes
import json
import os
import subprocess

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", default=os.path.join(ROOT, "build", "hbm_copy.so"))
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    if not os.path.exists(a.so):
        os.makedirs(os.path.dirname(a.so), exist_ok=True)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared",
                               "-fPIC", os.path.join(ROOT, "tools", "diag", "hbm_copy.hip"),
                               "-o", a.so])
    lib = ctypes.CDLL(a.so)
    lib.hbm_probe.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p] * 3 + [ctypes.c_int64,
                                                                         ctypes.c_void_p]
    dev = torch.device("cuda")
    n = 1 << 30    # bf16 elements: 2 GiB per operand
    A = torch.randn(n, device=dev, dtype=torch.bfloat16)
    B = torch.randn(n, device=dev, dtype=torch.bfloat16)
    C = torch.empty(n, device=dev, dtype=torch.bfloat16)
    n4 = n * 2 // 16
    st = torch.cuda.current_stream().cuda_stream

    def probe(kind, var, U, blocks):
        return lambda: lib.hbm_probe(kind, var, U, blocks, A.data_ptr(), B.data_ptr(),
                                     C.data_ptr(), n4, st)
    cases = []
    for kind, name, byt in ((0, "copy", 4 * n), (1, "add_2r1w", 6 * n), (2, "fill", 2 * n)):
        for var in ((0, 1, 2, 3) if kind == 0 else (0, 1)):
            for U in (1, 4, 8):
                for blocks in (0, 1024, 2048):
                    cases.append((f"{name}_v{var}_u{U}_g{blocks}", probe(kind, var, U, blocks), byt))
    cases += [("torch_copy", lambda: C.copy_(A), 4 * n),
              ("torch_add", lambda: torch.add(A, B, out=C), 6 * n),
              ("torch_fill", lambda: C.fill_(1.0), 2 * n)]
    ts = {c[0]: [] for c in cases}
    for _ in range(2):
        for _, f, _ in cases:
            f()
    torch.cuda.synchronize()
    for _ in range(a.reps):          # interleaved rounds
        for name, f, _ in cases:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            torch.cuda.synchronize()
            ts[name].append(e0.elapsed_time(e1) * 1e-3)
    for name, _, byt in cases:
        t = sorted(ts[name])[len(ts[name]) // 2]
        print(json.dumps({"case": name, "us": round(t * 1e6, 1), "tb_s": round(byt / t / 1e12, 3)}),
              flush=True)


if __name__ == "__main__":
    main()
