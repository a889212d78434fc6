#!/bin/bash
# Round 2, GPU pass 7: steady-state kernel profile of the default bench step with the fused
# conv + BN kernels (batch 2048).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/raw07 -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-baseline --virtual-workers 0 --profile-marker > $R/gpurun_out/r02_07_prof.log 2>&1 || { tail -20 $R/gpurun_out/r02_07_prof.log; exit 1; }
db=$(find $R/gpurun_out/raw07 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 70 --out $R/gpurun_out/r02_07_kernels.md
rm -rf $R/gpurun_out/raw07
head -5 $R/gpurun_out/r02_07_kernels.md
