#!/bin/bash
# Round 3, GPU pass 2: glds fused 1x1 kernels (conv1x1g.hip): bitwise A/B tests vs conv1x1.hip,
# per-shape A/B at the step's shapes, the existing fused-path tests, gossip k-mix kernel, and the
# step with the auto policy vs the old kernels (same box).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_02_*
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_conv1x1g_gpu.py tests/test_kernels_gpu.py -k "conv1x1g or gossip or test_bn_fwd or test_link or test_bnres or test_cat" > $O/r03_02_tests.log 2>&1 || { tail -40 $O/r03_02_tests.log; exit 1; }
tail -3 $O/r03_02_tests.log
timeout -k 10 300 python -u bench/conv1x1g.py > $O/r03_02_c1g.log 2>&1 || { tail -30 $O/r03_02_c1g.log; exit 1; }
cat $O/r03_02_c1g.log
timeout -k 10 500 $T tests/test_bwd_fusion_gpu.py tests/test_conv1x1_bn_gpu.py > $O/r03_02_fusion.log 2>&1 || { tail -40 $O/r03_02_fusion.log; exit 1; }
tail -3 $O/r03_02_fusion.log
timeout -k 10 300 python -u bench.py --no-baseline --virtual-workers 0 --b256-batch 0 > $O/r03_02_bench_auto.log 2>&1 || { tail -20 $O/r03_02_bench_auto.log; exit 1; }
grep '^{' $O/r03_02_bench_auto.log | cut -c1-300
CML_C1G=0 timeout -k 10 300 python -u bench.py --no-baseline --virtual-workers 0 --b256-batch 0 > $O/r03_02_bench_old.log 2>&1 || { tail -20 $O/r03_02_bench_old.log; exit 1; }
grep '^{' $O/r03_02_bench_old.log | cut -c1-300
