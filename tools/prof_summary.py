#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite) into a per-kernel table.

usage: python tools/prof_summary.py <run_results.db> [--top N] [--match REGEX] [--out file.md]
       [--after REGEX] [--steps K]

``--after REGEX`` keeps only dispatches that start after the LAST dispatch whose name matches
(bench.py --profile-marker launches a ``spin_kernel`` between warmup and the timed steps, so
``--after spin_kernel --steps K`` gives the steady-state per-step table without MIOpen find
trials or first-call work).
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
    ap.add_argument("--steps", type=int, default=0, help="also report ms per step over K steps")
    ap.add_argument("--after", default=None, help="window starts after the last match")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
    if a.after:
        rx_after = re.compile(a.after)
        marks = [e for name, s, e in rows if rx_after.search(name)]
        if marks:
            t0 = max(marks)
            rows = [r for r in rows if r[1] > t0 and not rx_after.search(r[0])]
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
    lines = [f"total kernel time: {total/1e3:.2f} ms over {sum(v[0] for v in agg.values())} dispatches"]
    K = max(a.steps, 0)
    if K:
        lines.append(f"per step (over {K} steps): {total/1e3/K:.2f} ms kernel time")
    if rows:
        # busy time = union of the dispatch intervals (overlapping kernels counted once); the rest
        # of the window's span is idle GPU time (launch gaps, host waits)
        iv = sorted((s_, e_) for _, s_, e_ in rows)
        busy, cs, ce = 0, iv[0][0], iv[0][1]
        for s_, e_ in iv[1:]:
            if s_ > ce:
                busy += ce - cs
                cs, ce = s_, e_
            else:
                ce = max(ce, e_)
        busy += ce - cs
        span = max(e_ for _, e_ in iv) - iv[0][0]
        lines.append(f"GPU busy {busy/1e6:.2f} ms of a {span/1e6:.2f} ms window "
                     f"({100 * busy / max(span, 1):.1f} %)")
    lines += ["", "| kernel | calls | total ms | avg us | % |" + (" ms/step |" if K else ""),
              "|---|---|---|---|---|" + ("---|" if K else "")]
    for name, (n, t) in items[: a.top]:
        short = re.sub(r"\s+", " ", name)[:110]
        extra = f" {t/1e3/K:.3f} |" if K else ""
        lines.append(f"| `{short}` | {n} | {t/1e3:.3f} | {t/n:.1f} | {100*t/total:.2f} |" + extra)
    text = "\n".join(lines)
    print(text)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(text + "\n")


if __name__ == "__main__":
    main()
