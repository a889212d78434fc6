#!/bin/bash
# Round 3, GPU pass 26 (re-run with the one-launch 3x3 weight layouts): stem backward with the pool input gradient gathered inside the stem weight-
# gradient kernel (stem_wgrad_pool): kernel tests, stem backward A/B at batch 2048, step A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_26_*
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_stem_gpu.py tests/test_conv3x3_layouts_gpu.py tests/test_conv1x1_bn_gpu.py tests/test_bwd_fusion_gpu.py > $O/r03_26_tests.txt 2>&1 || { tail -40 $O/r03_26_tests.txt; exit 1; }
tail -2 $O/r03_26_tests.txt
timeout -k 10 200 python -u bench/stem_bwd.py > $O/r03_26_stem.jsonl 2>&1 || { tail -20 $O/r03_26_stem.jsonl; exit 1; }
timeout -k 10 200 python -u bench/stem_bwd.py --dy2 >> $O/r03_26_stem.jsonl 2>&1 || { tail -20 $O/r03_26_stem.jsonl; exit 1; }
grep '^{' $O/r03_26_stem.jsonl
for arm in on off on off; do
  if [ $arm = on ]; then v=1; else v=0; fi
  CML_STEM_POOL_GATHER=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 4 --virtual-workers 0 --b256-batch 0 > $O/r03_26_bench_$arm.log 2>&1 || { tail -20 $O/r03_26_bench_$arm.log; exit 1; }
  echo "$arm $(grep -o '"ms_per_step": [0-9.]*' $O/r03_26_bench_$arm.log | head -1)" | tee -a $O/r03_26_ab.txt
done
