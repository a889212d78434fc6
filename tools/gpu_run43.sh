#!/bin/bash
# GPU pass 43: stem kernel timings + PMC counters of the weight-gradient kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
timeout -k 10 120 python tools/diag/stem_bench.py > gpurun_out/stem_bench43.log 2>&1 || exit $?
grep us gpurun_out/stem_bench43.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/pmc43a -o run -- python3 $R/tools/diag/stem_bench.py 64 > $R/gpurun_out/pmc43a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM_RD --output-format csv -d $R/gpurun_out/pmc43b -o run -- python3 $R/tools/diag/stem_bench.py 64 > $R/gpurun_out/pmc43b.log 2>&1 || exit $?
for d in pmc43a pmc43b; do f=$(find $R/gpurun_out/$d -name '*counter_collection.csv' -print -quit); python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:60]
    if "stem" not in k and "maxpool" not in k: continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    print(k, {c: round(v / cnt[(k, c)]) for c, v in d.items()})
PY
done
rm -rf $R/gpurun_out/pmc43a $R/gpurun_out/pmc43b
