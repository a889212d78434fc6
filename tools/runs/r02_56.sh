#!/bin/bash
# Round 2, GPU pass 56: cat-GEMM BN sums only on the 64-channel (layer-1) tails vs on every
# recompute tail vs off: step A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_56_*
for cfg in "1 64" "1 256" "0 64" "1 64" "1 256" "0 64"; do
set -- $cfg
CML_CAT_BNSUMS=$1 CML_CAT_BNSUMS_MAXC=$2 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_56_bench_$1_$2.log 2>&1 || { tail -20 $O/r02_56_bench_$1_$2.log; exit 1; }
echo "cat_bnsums=$1 maxc=$2 $(grep -o '"ms_per_step": [0-9.]*' $O/r02_56_bench_$1_$2.log)"
done
