#!/bin/bash
# Round 2, GPU pass 67: kernel profile of the final round-2 step (batch 2048).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_67_* $O/raw67
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw67 -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-baseline --virtual-workers 0 --profile-marker > $O/r02_67_prof.log 2>&1 || { tail -20 $O/r02_67_prof.log; exit 1; }
db=$(find $O/raw67 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 90 --out $O/r02_67_kernels.md
rm -rf $O/raw67
python3 $R/tools/kernel_classes.py $O/r02_67_kernels.md
