#!/usr/bin/env python3
"""HBM bytes per training step from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of a benchmark
started with --profile-marker: the dispatches after the marker kernel (``spin_kernel``) are the
timed steps. FETCH_SIZE is scaled by 2 (calibration: tools/pmc_summary.py) and both counters are
KiB per dispatch. Prints per-step GB read / written, per kernel class (tools/kernel_classes.py
rules) and in total, and the time floor at 6.3 TB/s (the measured float4-copy rate on MI355X).

  python tools/pmc_step_bytes.py --steps 3 DIR_FETCH DIR_WRITE
  python tools/pmc_step_bytes.py --steps 3 --per-kernel 40 DIR_FETCH DIR_WRITE

``--per-kernel N`` instead lists the N dispatch groups (kernel name + grid size) with the most
bytes: GB per step, ms per step (the counter run's own timestamps, so a little above a
kernel-trace run) and the achieved TB/s -- the kernels furthest from the copy rate.
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


def load_groups(d: str, counter: str):
    """{(kernel, grid): [counter sum, ns sum, calls]} after the marker."""
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    marker = max((int(r["Dispatch_Id"]) for r in rows if "spin_kernel" in r["Kernel_Name"]),
                 default=-1)
    out = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for r in rows:
        if int(r["Dispatch_Id"]) > marker and r["Counter_Name"] == counter:
            g = out[(r["Kernel_Name"], int(r["Grid_Size"]))]
            g[0] += float(r["Counter_Value"])
            g[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            g[2] += 1
    return out


def per_kernel(a) -> None:
    f = load_groups(a.fetch_dir, "FETCH_SIZE")
    w = load_groups(a.write_dir, "WRITE_SIZE")
    rows = []
    for key in set(f) | set(w):
        fr, wr = f.get(key, [0, 0, 0]), w.get(key, [0, 0, 0])
        gb = (2 * fr[0] + wr[0]) * 1024 / 1e9 / a.steps
        ms = max(fr[1], wr[1]) / 1e6 / a.steps
        rows.append((gb, ms, max(fr[2], wr[2]) // a.steps, key))
    rows.sort(key=lambda r: -r[0])
    print("| kernel | grid | calls / step | GB / step | ms / step | TB/s |")
    print("|---|---|---|---|---|---|")
    for gb, ms, calls, (name, grid) in rows[:a.per_kernel]:
        print(f"| `{name[:90]}` | {grid} | {calls} | {gb:.2f} | {ms:.3f} | "
              f"{gb / ms if ms else 0:.2f} |")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--per-kernel", type=int, default=0)
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    a = ap.parse_args()
    if a.per_kernel:
        return per_kernel(a)
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
