#!/bin/bash
# Round 3, GPU pass 31: stride-2 3x3 convs on conv_gemm.hip (parity-class data gradient + bn1 sums):
# new tests, per-shape timing vs MIOpen (batch 2048 and 256), step A/B (own_conv3x3_s2 on / off),
# then the full GPU suite and the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_31_*
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv3x3_s2_gpu.py > $O/r03_31_tests.txt 2>&1 || { tail -40 $O/r03_31_tests.txt; exit 1; }
tail -2 $O/r03_31_tests.txt
timeout -k 10 200 python -u bench/conv3x3_s2.py --batch 256 > $O/r03_31_shapes.jsonl 2>&1 || { tail -20 $O/r03_31_shapes.jsonl; exit 1; }
timeout -k 10 200 python -u bench/conv3x3_s2.py --batch 2048 >> $O/r03_31_shapes.jsonl 2>&1 || { tail -20 $O/r03_31_shapes.jsonl; exit 1; }
grep '^{' $O/r03_31_shapes.jsonl
for rep in 1 2; do
  for arm in default nos2; do
    case $arm in
      default) envs="";;
      nos2) envs="CML_CONV3X3_S2=0";;
    esac
    env $envs timeout -k 10 300 python -u bench.py --steps 10 --warmup 4 --no-baseline --virtual-workers 0 --b256-batch 0 > $O/r03_31_bench_$arm$rep.log 2>&1 || { tail -20 $O/r03_31_bench_$arm$rep.log; exit 1; }
    echo "$arm $rep $(grep -o '"ms_per_step": [0-9.]*' $O/r03_31_bench_$arm$rep.log | head -1)" | tee -a $O/r03_31_ab.txt
  done
done
for arm in default nos2; do
  case $arm in
    default) envs="";;
    nos2) envs="CML_CONV3X3_S2=0";;
  esac
  env $envs timeout -k 10 300 python -u bench.py --batch 256 --steps 30 --warmup 5 --no-baseline --virtual-workers 0 --b256-batch 0 > $O/r03_31_b256_$arm.log 2>&1 || { tail -20 $O/r03_31_b256_$arm.log; exit 1; }
  echo "b256 $arm $(grep -o '"ms_per_step": [0-9.]*' $O/r03_31_b256_$arm.log | head -1)" | tee -a $O/r03_31_ab.txt
done
timeout -k 10 900 python -u -m pytest tests -m gpu --deselect tests/test_convergence_gpu.py::test_fused_step_trains_like_library -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/r03_31_gputests.txt 2>&1 || { tail -40 $O/r03_31_gputests.txt; exit 1; }
tail -2 $O/r03_31_gputests.txt
timeout -k 10 600 python -u bench.py > $O/r03_31_bench.log 2>&1 || { tail -30 $O/r03_31_bench.log; exit 1; }
grep '"metric"' $O/r03_31_bench.log > $O/r03_31_bench.json; cut -c1-400 $O/r03_31_bench.json
