#!/bin/bash
# Round 2, GPU pass 46: recompute-tail policy with Gram statistics -- layer 4 (512 planes) on / off.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_46_*
for p in 256 512 256 512; do
CML_RECOMPUTE_TAIL_MAX_PLANES=$p timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_46_bench$p.log 2>&1 || { tail -20 $O/r02_46_bench$p.log; exit 1; }
echo "max_planes=$p $(grep -o '"ms_per_step": [0-9.]*' $O/r02_46_bench$p.log)"
done
