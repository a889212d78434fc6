#!/bin/bash
# Round 3, GPU pass 33: layer-4 stride-2 downsample as a stride-1 GEMM of x[:, :, ::2, ::2] with its
# compact data gradient parked on conv1's link (PerfPolicy.down_s2_compact): tests, step A/B at
# batch 2048 and 256.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_33_*
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv3x3_s2_gpu.py > $O/r03_33_tests.txt 2>&1 || { tail -40 $O/r03_33_tests.txt; exit 1; }
tail -2 $O/r03_33_tests.txt
for rep in 1 2; do
  for arm in default nocompact; do
    case $arm in
      default) envs="";;
      nocompact) envs="CML_DOWN_S2_COMPACT=0";;
    esac
    env $envs timeout -k 10 300 python -u bench.py --steps 10 --warmup 4 --no-baseline --virtual-workers 0 --b256-batch 0 > $O/r03_33_bench_$arm$rep.log 2>&1 || { tail -20 $O/r03_33_bench_$arm$rep.log; exit 1; }
    echo "$arm $rep $(grep -o '"ms_per_step": [0-9.]*' $O/r03_33_bench_$arm$rep.log | head -1)" | tee -a $O/r03_33_ab.txt
    env $envs timeout -k 10 300 python -u bench.py --batch 256 --steps 30 --warmup 5 --no-baseline --virtual-workers 0 --b256-batch 0 > $O/r03_33_b256_$arm$rep.log 2>&1 || { tail -20 $O/r03_33_b256_$arm$rep.log; exit 1; }
    echo "b256 $arm $rep $(grep -o '"ms_per_step": [0-9.]*' $O/r03_33_b256_$arm$rep.log | head -1)" | tee -a $O/r03_33_ab.txt
  done
done
