#!/bin/bash
# r06 pass 34: batch-256 kernel table + classes on the current code (VERDICT item 7 evidence).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_34; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --batch 256 --steps 10 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 400 --out $O/kernels_b256.md > /dev/null
rm -rf $O/raw
python3 $R/tools/kernel_classes.py $O/kernels_b256.md > $O/classes_b256.md
head -3 $O/kernels_b256.md
cat $O/classes_b256.md
