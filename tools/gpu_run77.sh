#!/bin/bash
# GPU pass 77: steady-state kernel profile of the final round-1 kernels at the default batch 2048.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/raw77 -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-baseline --profile-marker > $R/gpurun_out/prof77.log 2>&1 || exit $?
db=$(find $R/gpurun_out/raw77 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 60 --out $R/gpurun_out/prof77_resnet_kernels.md
rm -rf $R/gpurun_out/raw77
tail -1 $R/gpurun_out/prof77.log | cut -c1-200
