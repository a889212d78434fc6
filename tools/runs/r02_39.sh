#!/bin/bash
# Round 2, GPU pass 39: nine-tap 3x3 weight-gradient kernel (wgrad3x3.hip): numerics vs fp32, then
# per-shape timing vs MIOpen and the TAP kernel at batch 2048.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_39_*
timeout -k 10 300 python -u -m pytest tests/test_conv1x1_bn_gpu.py -k wgrad3x3 -x -v --timeout 120 --timeout-method thread > $O/r02_39_pytest.log 2>&1 || { tail -40 $O/r02_39_pytest.log; exit 1; }
tail -3 $O/r02_39_pytest.log
timeout -k 10 300 python -u bench/wgrad3x3.py --json-out $O/r02_39_wgrad3x3.jsonl > $O/r02_39_bench.log 2>&1 || { tail -20 $O/r02_39_bench.log; exit 1; }
cat $O/r02_39_bench.log
