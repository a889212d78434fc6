#!/usr/bin/env python3
"""Per-kernel VGPR / AGPR / spill / occupancy / LDS table of HIP sources (gfx950), from the
compiler's kernel-resource-usage remarks:  python tools/kernel_resources.py csrc/kernels/gram.hip"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def table(src):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I",
           os.path.join(ROOT, "csrc"), "-c", src, "-o", "/tmp/_kr.o",
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    return rows


if __name__ == "__main__":
    for src in sys.argv[1:]:
        for r in table(src):
            g = r.get
            print(f"{g('VGPRs', '?'):>4} vgpr {g('AGPRs', '?'):>4} agpr  spill {g('VGPRs Spill', '?'):>4}"
                  f"  occ {g('Occupancy [waves/SIMD]', '?'):>2}  lds {g('LDS Size [bytes/block]', '?'):>6}"
                  f"  {r['name']}")
