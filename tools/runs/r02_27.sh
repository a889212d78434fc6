#!/bin/bash
# Round 2, GPU pass 27: wgrad3x3 tests + 1x1 data-gradient GEMMs conv_gemm vs hipBLASLt.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv1x1_bn_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "wgrad3x3 or conv_gemm" > $O/r02_27_pytest.log 2>&1 || { tail -30 $O/r02_27_pytest.log; exit 1; }
tail -1 $O/r02_27_pytest.log
timeout -k 10 300 python -u bench/gemm1x1.py > $O/r02_27_gemm1x1.jsonl 2>$O/r02_27.err || { tail -20 $O/r02_27.err; exit 1; }
cat $O/r02_27_gemm1x1.jsonl
