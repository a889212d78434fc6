#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite) into a per-kernel table.

usage: python tools/prof_summary.py <run_results.db> [--top N] [--match REGEX] [--out file.md]
"""
import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--match", default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--steps", type=int, default=0, help="divide totals by this many steps")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
    agg = {}
    for name, s, e in rows:
        d = agg.setdefault(name, [0, 0.0])
        d[0] += 1
        d[1] += (e - s) / 1e3   # ns -> us
    total = sum(v[1] for v in agg.values())
    items = sorted(agg.items(), key=lambda kv: -kv[1][1])
    if a.match:
        rx = re.compile(a.match)
        items = [kv for kv in items if rx.search(kv[0])]
    lines = [f"total kernel time: {total/1e3:.2f} ms over {sum(v[0] for v in agg.values())} dispatches",
             "", "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for name, (n, t) in items[: a.top]:
        short = re.sub(r"\s+", " ", name)[:110]
        lines.append(f"| `{short}` | {n} | {t/1e3:.3f} | {t/n:.1f} | {100*t/total:.2f} |")
    text = "\n".join(lines)
    print(text)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(text + "\n")


if __name__ == "__main__":
    main()
