#!/usr/bin/env python3
"""Kernels with exactly known HBM traffic, for calibrating rocprofv3's FETCH_SIZE / WRITE_SIZE.

Working sets from 64 MiB (inside the 256 MiB MALL / Infinity Cache) to 2000 MiB (far outside it;
larger tensors make PyTorch split an op into several launches, which the matcher would miss):
  copy   dst.copy_(src)     bf16, reads N bytes, writes N bytes
  sum    src.sum()          bf16 -> fp32 scalar, reads N bytes
  cast   dst16.copy_(src32) fp32 -> bf16, reads N bytes, writes N / 2 bytes
Each op runs 3 times after its inputs are produced by a fill; the dispatch order is written to
``--manifest`` (JSON) for tools/diag/fetch_calibration_report.py, which matches it against the
counter CSVs of two runs (FETCH_SIZE pass, WRITE_SIZE pass):

  rocprofv3 --pmc FETCH_SIZE -d gpurun_out/cal_f -o run -- python tools/diag/fetch_calibration.py
  rocprofv3 --pmc WRITE_SIZE -d gpurun_out/cal_w -o run -- python tools/diag/fetch_calibration.py
"""
import argparse
import json

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--manifest", default=None)
    ap.add_argument("--sizes-mib", default="64,1024,2000")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    man = []
    for mib in [int(s) for s in a.sizes_mib.split(",")]:
        nbytes = mib << 20
        src = torch.empty(nbytes // 2, dtype=torch.bfloat16, device=dev).fill_(1.0)
        dst = torch.empty_like(src)
        torch.cuda.synchronize()
        for _ in range(3):
            dst.copy_(src)
            man.append({"op": "copy", "mib": mib, "read": nbytes, "write": nbytes,
                        "pattern": "copy|elementwise"})
        for _ in range(3):
            src.sum()
            man.append({"op": "sum", "mib": mib, "read": nbytes, "write": 0,
                        "pattern": "reduce"})
        del dst
        s32 = torch.empty(nbytes // 4, dtype=torch.float32, device=dev).fill_(1.0)
        d16 = torch.empty(nbytes // 4, dtype=torch.bfloat16, device=dev)
        torch.cuda.synchronize()
        for _ in range(3):
            d16.copy_(s32)
            man.append({"op": "cast_f32_bf16", "mib": mib, "read": nbytes, "write": nbytes // 2,
                        "pattern": "copy|elementwise"})
        torch.cuda.synchronize()
        del src, s32, d16
        torch.cuda.empty_cache()
    if a.manifest:
        with open(a.manifest, "w") as fh:
            json.dump(man, fh, indent=1)
    print("ops", len(man))


if __name__ == "__main__":
    main()
