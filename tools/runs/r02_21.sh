#!/bin/bash
# Round 2, GPU pass 21: 3x3 implicit-GEMM experiment vs MIOpen + bench contract tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -f $O/r02_21_*
timeout -k 10 400 python -u bench/conv3x3.py > $O/r02_21_conv3x3.jsonl 2>$O/r02_21.err || { tail -20 $O/r02_21.err; exit 1; }
cat $O/r02_21_conv3x3.jsonl
timeout -k 10 900 python -u -m pytest tests/test_bench_contract_gpu.py -m gpu -x -q --timeout 850 --timeout-method thread > $O/r02_21_pytest.log 2>&1 || { tail -30 $O/r02_21_pytest.log; exit 1; }
tail -1 $O/r02_21_pytest.log
