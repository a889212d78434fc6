#!/bin/bash
# Round 2, GPU pass 61: batch-256 step -- kernel time per step vs wall time (launch gaps?).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_61_* $O/raw61
timeout -k 10 300 python -u bench.py --batch 256 --steps 30 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_61_bench.log 2>&1 || { tail -20 $O/r02_61_bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/r02_61_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/raw61 -o run -- python3 $R/bench.py --batch 256 --steps 10 --warmup 3 --no-baseline --virtual-workers 0 --profile-marker > $O/r02_61_prof.log 2>&1 || { tail -20 $O/r02_61_prof.log; exit 1; }
db=$(find $O/raw61 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 40 --out $O/r02_61_kernels.md
rm -rf $O/raw61
grep -E "per step|total kernel" $O/r02_61_kernels.md
