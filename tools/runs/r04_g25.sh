#!/bin/bash
# Round 4, GPU pass 25: held clock and MFMA-pipe busy share of the layer-1 3x3 kernels
# (GRBM_GUI_ACTIVE / 8 / wall = effective clock; SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles)).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_25}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  CML_CONV3P=$v timeout -s KILL 90 rocprofv3 --output-format csv --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d $O/pmc_$v -o run -- python3 $R/bench/conv3x3p.py --reps 5 > $O/pmc_$v.log 2>&1 || { tail -20 $O/pmc_$v.log; exit 1; }
  python3 - $O/pmc_$v/run_counter_collection.csv $v <<'PY' >> $O/clock.md
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r["Kernel_Name"]
    if not ("conv3x3p" in k or "conv_gemm_kernel" in k):
        continue
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg[k[:70]][r["Counter_Name"]].append((float(r["Counter_Value"]), dur))
for k, d in agg.items():
    g = d["GRBM_GUI_ACTIVE"]
    m = d["SQ_VALU_MFMA_BUSY_CYCLES"]
    n = len(g)
    clk = sum(v / 8 / t for v, t in g) / n / 1e9
    cyc = sum(v / 8 for v, t in g) / n
    mf = sum(v for v, t in m) / len(m)
    print(f"| CML_CONV3P={sys.argv[2]} | `{k}` | {n} | {sum(t for v, t in g) / n * 1e3:.3f} | {clk:.2f} | {100 * mf / (1024 * cyc):.1f} |")
PY
  find $O/pmc_$v -type f ! -name 'run_counter_collection.csv' -delete
done
cat $O/clock.md
