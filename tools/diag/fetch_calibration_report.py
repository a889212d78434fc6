#!/usr/bin/env python3
"""Match fetch_calibration.py's manifest against rocprofv3 counter CSVs and report the ratio of
counted to true bytes per op and working-set size (markdown).

  python tools/diag/fetch_calibration_report.py manifest.json gpurun_out/cal_f gpurun_out/cal_w
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def load(d):
    hits = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not hits:
        raise FileNotFoundError(f"no counter_collection.csv under {d}")
    path = hits[0]
    rows = {}
    for r in csv.DictReader(open(path)):
        did = int(r["Dispatch_Id"])
        e = rows.setdefault(did, {"name": r["Kernel_Name"], "c": collections.defaultdict(float)})
        e["c"][r["Counter_Name"]] += float(r["Counter_Value"])
    return [rows[k] for k in sorted(rows)]


def match(man, disp):
    out, k = [], 0
    for m in man:
        pat = re.compile(m["pattern"], re.I)
        while k < len(disp) and not (pat.search(disp[k]["name"]) and "fill" not in disp[k]["name"].lower()):
            k += 1
        out.append(disp[k] if k < len(disp) else None)
        k += 1
    return out


def main(manifest, fdir, wdir):
    man = json.load(open(manifest))
    f = match(man, load(fdir))
    w = match(man, load(wdir))
    agg = collections.defaultdict(list)
    for m, fe, we in zip(man, f, w):
        fr = fe["c"].get("FETCH_SIZE", 0) * 1024 / m["read"] if fe and m["read"] else None
        wr = we["c"].get("WRITE_SIZE", 0) * 1024 / m["write"] if we and m["write"] else None
        agg[(m["op"], m["mib"])].append((fr, wr))
    print("| op | working set MiB | FETCH_SIZE x 1 KiB / true bytes read | WRITE_SIZE x 1 KiB / true bytes written |")
    print("|---|---|---|---|")
    for (op, mib), v in agg.items():
        fs = [x for x, _ in v if x is not None]
        ws = [y for _, y in v if y is not None]
        fcell = " / ".join(f"{x:.3f}" for x in fs) or "-"
        wcell = " / ".join(f"{y:.3f}" for y in ws) or "-"
        print(f"| {op} | {mib} | {fcell} | {wcell} |")


if __name__ == "__main__":
    main(*sys.argv[1:4])
