#!/bin/bash
# Round 3, GPU pass 29: both stem backward paths stage g itself (mean(g) through the column sums of the
# input patches, vectorised column-sum pass): tests, gather-vs-two-pass-vs-fp64 over
# batch sizes, stem backward timing at batch 2048, step A/B (gather on / off).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_29_*
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_stem_gpu.py tests/test_conv3x3_layouts_gpu.py tests/test_bwd_fusion_gpu.py > $O/r03_29_tests.txt 2>&1 || { tail -40 $O/r03_29_tests.txt; exit 1; }
tail -2 $O/r03_29_tests.txt
timeout -k 10 400 python -u tools/diag/stem_gather_diag.py > $O/r03_29_diag.jsonl 2>&1 || { tail -30 $O/r03_29_diag.jsonl; exit 1; }
grep '^{' $O/r03_29_diag.jsonl
timeout -k 10 200 python -u bench/stem_bwd.py > $O/r03_29_stem.jsonl 2>&1 || { tail -20 $O/r03_29_stem.jsonl; exit 1; }
timeout -k 10 200 python -u bench/stem_bwd.py --dy2 >> $O/r03_29_stem.jsonl 2>&1 || { tail -20 $O/r03_29_stem.jsonl; exit 1; }
grep '^{' $O/r03_29_stem.jsonl
for rep in 1 2; do
  for arm in default nogather; do
    case $arm in
      default) envs="";;
      nogather) envs="CML_STEM_POOL_GATHER=0";;
    esac
    env $envs timeout -k 10 300 python -u bench.py --steps 10 --warmup 4 --no-baseline --virtual-workers 0 --b256-batch 0 > $O/r03_29_bench_$arm$rep.log 2>&1 || { tail -20 $O/r03_29_bench_$arm$rep.log; exit 1; }
    echo "$arm $rep $(grep -o '"ms_per_step": [0-9.]*' $O/r03_29_bench_$arm$rep.log | head -1)" | tee -a $O/r03_29_ab.txt
  done
done
