#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc runs (one counter group per run) into one per-kernel markdown table.

  python tools/pmc_summary.py gpurun_out/pmc7_fetch_size gpurun_out/pmc7_write_size \
      gpurun_out/pmc7_sq_insts_valu_mfma_mops_bf16 > profiles/xxx_pmc.md

Per kernel: dispatches, mean duration (from the counter run's own timestamps), mean counter
values, and derived HBM-side rates: FETCH_SIZE / WRITE_SIZE are KiB per dispatch -> GB/s over the
dispatch duration; SQ_INSTS_VALU_MFMA_MOPS_BF16 counts 512-FLOP units -> TFLOP/s. Derived against
the MI355X peaks: HBM % = (scaled fetch + write) bytes / duration / 8 TB/s, MFMA % = bf16 MFMA
FLOP / duration / 2.5 PFLOP/s (dense), and the effective clock GRBM_GUI_ACTIVE / 8 / duration
(the counter sums the 8 XCDs; reads high on dispatches under ~0.3 ms).

Calibration on this MI355X image (tools/diag/fetch_calibration.py, profiles/
r02_fetch_size_calibration.md): on kernels with exactly known traffic -- a bf16 copy, a bf16 sum
and an fp32->bf16 cast at 64 MiB (inside the 256 MiB MALL), 1 GiB and 2000 MiB working sets --
FETCH_SIZE x 1 KiB is 0.500 of the true bytes read in every case (not a cache effect) and
WRITE_SIZE is exact, so ``--fetch-scale 2`` (default) is applied to the fetch rate; the raw
counter column is unscaled.
"""
import collections
import csv
import os
import re
import sys


def short(name: str) -> str:
    name = name.replace("void ", "").replace("(anonymous namespace)::", "").replace("cml::", "")
    name = re.sub(r"\(.*", "", name)
    return name[:70]


def main(dirs, fetch_scale=2.0, match=None):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for d in dirs:
        path = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            if match is not None and not re.search(match, k):
                continue
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[(k, d, r["Dispatch_Id"])] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    kd = collections.defaultdict(list)
    for (k, _, _), v in dur.items():
        kd[k].append(v)
    counters = sorted({c for k in acc for c in acc[k]})
    print("| kernel | dispatches | mean us | " + " | ".join(counters) +
          " | fetch GB/s | write GB/s | bf16 MFMA TFLOP/s | HBM % of 8 TB/s | MFMA % of 2.5 PF | clock GHz |")
    print("|---|---|---|" + "---|" * len(counters) + "---|---|---|---|---|---|")
    for k in sorted(kd, key=lambda k: -sum(kd[k])):
        us = sum(kd[k]) / len(kd[k]) / 1e3
        mean = {c: sum(v) / len(v) for c, v in acc[k].items()}
        cells = [f"{mean[c]:.4g}" if c in mean else "" for c in counters]
        fetch = mean.get("FETCH_SIZE")
        write = mean.get("WRITE_SIZE")
        mops = mean.get("SQ_INSTS_VALU_MFMA_MOPS_BF16")
        rate = lambda kib, sc=1.0: (f"{sc * kib * 1024 / (us * 1e-6) / 1e9:.0f}"
                                    if kib is not None and us > 0 else "")
        tf = f"{mops * 512 / (us * 1e-6) / 1e12:.1f}" if mops is not None and us > 0 else ""
        hbm = ""
        if (fetch is not None or write is not None) and us > 0:
            by = fetch_scale * (fetch or 0.0) * 1024 + (write or 0.0) * 1024
            hbm = f"{100 * by / (us * 1e-6) / 8e12:.1f}"
        mf = f"{100 * mops * 512 / (us * 1e-6) / 2.5e15:.1f}" if mops is not None and us > 0 else ""
        gui = mean.get("GRBM_GUI_ACTIVE")
        clk = f"{gui / 8 / (us * 1e-6) / 1e9:.2f}" if gui is not None and us > 0 else ""
        print(f"| `{k}` | {len(kd[k]) // max(1, len(dirs))} | {us:.1f} | " +
              " | ".join(cells) + f" | {rate(fetch, fetch_scale)} | {rate(write)} | {tf} | {hbm} | {mf} | {clk} |")


if __name__ == "__main__":
    args = sys.argv[1:]
    scale = 2.0
    if "--fetch-scale" in args:
        i = args.index("--fetch-scale")
        scale = float(args[i + 1])
        del args[i:i + 2]
    match = None
    if "--match" in args:
        i = args.index("--match")
        match = args[i + 1]
        del args[i:i + 2]
    main(args, scale, match)
