#!/bin/bash
# Round 4, GPU pass 21: batch-256 step profile (launch count, GPU-busy share, kernel classes).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_21}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --batch 256 --steps 10 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 400 --out $O/kernels_b256.md
python3 $R/tools/kernel_classes.py $O/kernels_b256.md > $O/classes_b256.md || true
rm -rf $O/raw
grep -i "busy\|dispatches\|per step" $O/kernels_b256.md | head
cat $O/classes_b256.md
