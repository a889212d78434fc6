#!/usr/bin/env python3
"""HBM bytes per training step from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of a benchmark
started with --profile-marker: the dispatches after the marker kernel (``spin_kernel``) are the
timed steps. FETCH_SIZE is scaled by 2 (calibration: tools/pmc_summary.py) and both counters are
KiB per dispatch. Prints per-step GB read / written, per kernel class (tools/kernel_classes.py
rules) and in total, and the time floor at 6.3 TB/s (the measured float4-copy rate on MI355X).

  python tools/pmc_step_bytes.py --steps 3 DIR_FETCH DIR_WRITE
"""
import argparse
import collections
import csv
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_classes import CLASSES  # noqa: E402


def classify(name: str) -> str:
    for cls, pat in CLASSES:
        if re.search(pat, name):
            return cls
    return "other (fills, copies, elementwise)"


def load(d: str, counter: str):
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    marker = max((int(r["Dispatch_Id"]) for r in rows if "spin_kernel" in r["Kernel_Name"]),
                 default=-1)
    out = collections.defaultdict(float)
    for r in rows:
        if int(r["Dispatch_Id"]) > marker and r["Counter_Name"] == counter:
            out[classify(r["Kernel_Name"])] += float(r["Counter_Value"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    a = ap.parse_args()
    f = load(a.fetch_dir, "FETCH_SIZE")
    w = load(a.write_dir, "WRITE_SIZE")
    gb = lambda kib: kib * 1024 / 1e9 / a.steps
    print("| class | read GB / step | written GB / step | total GB / step | floor ms at 6.3 TB/s |")
    print("|---|---|---|---|---|")
    tot_r = tot_w = 0.0
    for cls in sorted(set(f) | set(w), key=lambda c: -(2 * f.get(c, 0) + w.get(c, 0))):
        r, wr = gb(2 * f.get(cls, 0.0)), gb(w.get(cls, 0.0))
        tot_r += r
        tot_w += wr
        print(f"| {cls} | {r:.1f} | {wr:.1f} | {r + wr:.1f} | {(r + wr) / 6.3:.2f} |")
    print(f"| total | {tot_r:.1f} | {tot_w:.1f} | {tot_r + tot_w:.1f} | "
          f"{(tot_r + tot_w) / 6.3:.2f} |")


if __name__ == "__main__":
    main()
