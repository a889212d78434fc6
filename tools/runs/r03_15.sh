#!/bin/bash
# Round 3, GPU pass 15: bn_stats_gram at 8 channels per workgroup with 16 float4 loads in flight;
# tail_prep.hip with LDS-staged tiles, split-K partials of G and a third (sum) launch. Fusion tests, bench (batch 2048 and 256), kernel profiles
# of the two batch sizes (b256 block off so the profile holds only the measured step).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_15_* $O/raw15*
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bwd_fusion_gpu.py tests/test_conv1x1g_gpu.py tests/test_conv1x1_bn_gpu.py > $O/r03_15_tests.txt 2>&1 || { tail -40 $O/r03_15_tests.txt; exit 1; }
tail -2 $O/r03_15_tests.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --b256-batch 0 > $O/r03_15_bench.log 2>&1 || { tail -30 $O/r03_15_bench.log; exit 1; }
grep '"metric"' $O/r03_15_bench.log | cut -c1-300
timeout -k 10 300 python -u bench.py --batch 256 --steps 30 --warmup 5 --no-baseline --virtual-workers 0 > $O/r03_15_b256.log 2>&1 || { tail -30 $O/r03_15_b256.log; exit 1; }
grep '"metric"' $O/r03_15_b256.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
for B in 2048 256; do
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw15_$B -o run -- python3 $R/bench.py --batch $B --steps 6 --warmup 2 --no-baseline --virtual-workers 0 --b256-batch 0 --profile-marker > $O/r03_15_prof$B.log 2>&1 || { tail -20 $O/r03_15_prof$B.log; exit 1; }
db=$(find $O/raw15_$B -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 100 --out $O/r03_15_kernels_b$B.md
rm -rf $O/raw15_$B
python3 $R/tools/kernel_classes.py $O/r03_15_kernels_b$B.md | tee $O/r03_15_classes_b$B.md
done
