#!/bin/bash
# r06 pass 1: gemm_w4.hip (4-wave 256 x 256 tiles, any operand layout) numerics vs fp32, then its
# square / Llama shapes vs hipBLASLt and gemm.hip.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_01; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_w4_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench/gemm_w4.py --json-out $O/gemm_w4.jsonl > $O/gemm_w4.log 2>&1 || { tail -20 $O/gemm_w4.log; exit 1; }
cut -c1-400 $O/gemm_w4.jsonl
