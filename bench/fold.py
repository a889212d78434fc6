"""Split-K fold timing (wgrad1x1.hip fold_splits) at the slab shapes the ResNet-50 weight gradients
produce; run twice, with CML_FOLD_WIDE_MIN=0 (narrow kernel only) and the default, for the A/B."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from consensusml_amd.ops.native import lib

SHAPES = [(2048, 4096), (2048, 64), (512, 16384), (512, 256), (128, 65536), (128, 1024),
          (32, 262144), (8, 1048576), (16, 2359296)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rows = []
    for S, n in SHAPES:
        part = torch.randn(S, n, device=dev)
        for _ in range(3):
            lib().split_fold(part, False)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            lib().split_fold(part, False)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        r = {"S": S, "n": n, "us": round(us, 2), "GBps": round(S * n * 4 / us / 1e3, 1),
             "wide_min": os.environ.get("CML_FOLD_WIDE_MIN", "32")}
        rows.append(r)
        print(json.dumps(r), flush=True)
    if a.json_out:
        with open(a.json_out, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
