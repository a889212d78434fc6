#!/bin/bash
# Round 2, GPU pass 2: fused 1x1 conv + BN statistics kernel: numerics, then per-shape timing.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv1x1_bn_gpu.py tests/test_wgrad1x1_gpu.py -x -q --timeout 120 --timeout-method thread > $O/r02_03_pytest.log 2>&1 || { tail -40 $O/r02_03_pytest.log; exit 1; }
tail -3 $O/r02_03_pytest.log
timeout -k 10 300 python -u bench/conv1x1_fused.py --batch 2048 --json-out $O/r02_03_conv1x1.jsonl > $O/r02_03_bench.log 2>&1 || { tail -20 $O/r02_03_bench.log; exit 1; }
cat $O/r02_03_bench.log | cut -c1-400
