#!/bin/bash
# r06 pass 66: batch-2560 kernel table on the final code (library kernels left).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_66; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --steps 6 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 400 --out $O/kernels_b2560.md > /dev/null
rm -rf $O/raw
python3 $R/tools/kernel_classes.py $O/kernels_b2560.md > $O/classes_b2560.md
head -3 $O/kernels_b2560.md
cat $O/classes_b2560.md
