#!/bin/bash
# Round 2, GPU pass 13: backward-fusion kernels (BN-backward prologue / masked-link epilogue /
# coefficients / wgrad dz prologue) vs fp32 oracles, fused vs unfused identity chains, the
# whole-model fused test, then the bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -f $O/r02_13_*
timeout -k 10 400 python -u -m pytest tests/test_bwd_fusion_gpu.py tests/test_conv1x1_bn_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/r02_13_pytest.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/r02_13_pytest.log | tail -30; tail -40 $O/r02_13_pytest.log; exit 1; }
grep -cE "PASSED" $O/r02_13_pytest.log; tail -1 $O/r02_13_pytest.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/r02_13_bench.log 2>&1 || { tail -20 $O/r02_13_bench.log; exit 1; }
grep '"metric"' $O/r02_13_bench.log | cut -c1-700
