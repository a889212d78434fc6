#!/bin/bash
# Round 3, GPU pass 37: the four parity classes of the stride-2 data gradient in one launch
# (t = 4 tile + class, CML_S2DGRAD_ONE): conv tests, per-shape timing one vs four launches, step A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_37_*
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv3x3_s2_gpu.py tests/test_bwd_fusion_gpu.py tests/test_conv1x1_bn_gpu.py tests/test_conv3x3_layouts_gpu.py > $O/r03_37_tests.txt 2>&1 || { tail -40 $O/r03_37_tests.txt; exit 1; }
tail -2 $O/r03_37_tests.txt
for one in 1 0; do
  for B in 256 2048; do
    CML_S2DGRAD_ONE=$one timeout -k 10 200 python -u bench/conv3x3_s2.py --batch $B > $O/r03_37_shapes_one${one}_b$B.jsonl 2>&1 || { tail -20 $O/r03_37_shapes_one${one}_b$B.jsonl; exit 1; }
    grep '^{' $O/r03_37_shapes_one${one}_b$B.jsonl | cut -c1-200
  done
done
for rep in 1 2; do
  for one in 1 0; do
    CML_S2DGRAD_ONE=$one timeout -k 10 300 python -u bench.py --steps 10 --warmup 4 --no-baseline --virtual-workers 0 --b256-batch 0 > $O/r03_37_bench_one$one$rep.log 2>&1 || { tail -20 $O/r03_37_bench_one$one$rep.log; exit 1; }
    echo "one=$one $rep $(grep -o '"ms_per_step": [0-9.]*' $O/r03_37_bench_one$one$rep.log | head -1)" | tee -a $O/r03_37_ab.txt
  done
done
