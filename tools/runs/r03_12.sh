#!/bin/bash
# Round 3, GPU pass 12: auto policy = the persistent kernel for every fused 1x1 GEMM except the
# downsample tails' forward (quad). Fused-kernel tests, default bench, kernel profile of the step
# (batch 2048) and of batch 256.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_12_* $O/raw12*
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bwd_fusion_gpu.py tests/test_conv1x1g_gpu.py tests/test_conv1x1_bn_gpu.py > $O/r03_12_tests.txt 2>&1 || { tail -40 $O/r03_12_tests.txt; exit 1; }
tail -2 $O/r03_12_tests.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/r03_12_bench.log 2>&1 || { tail -30 $O/r03_12_bench.log; exit 1; }
grep '"metric"' $O/r03_12_bench.log > $O/r03_12_bench.json; cut -c1-400 $O/r03_12_bench.json
timeout -k 10 300 python -u bench.py --batch 256 --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r03_12_b256.log 2>&1 || { tail -30 $O/r03_12_b256.log; exit 1; }
grep '"metric"' $O/r03_12_b256.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw12 -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-baseline --virtual-workers 0 --profile-marker > $O/r03_12_prof.log 2>&1 || { tail -20 $O/r03_12_prof.log; exit 1; }
db=$(find $O/raw12 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 90 --out $O/r03_12_kernels.md
rm -rf $O/raw12
python3 $R/tools/kernel_classes.py $O/r03_12_kernels.md | tee $O/r03_12_classes.md
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw12b -o run -- python3 $R/bench.py --batch 256 --steps 10 --warmup 3 --no-baseline --virtual-workers 0 --profile-marker > $O/r03_12_profb.log 2>&1 || { tail -20 $O/r03_12_profb.log; exit 1; }
db=$(find $O/raw12b -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 90 --out $O/r03_12_kernels_b256.md
rm -rf $O/raw12b
python3 $R/tools/kernel_classes.py $O/r03_12_kernels_b256.md | tee $O/r03_12_classes_b256.md
