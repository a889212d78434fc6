#!/bin/bash
# Round 3, GPU pass 1: baseline of the round-2 state on this round's boxes: per-shape 1x1 conv
# timings (fused kernel vs library, conv_gemm taps=1 vs hipBLASLt) and the default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_01_*
timeout -k 10 300 python -u bench/conv1x1_fused.py --batch 2048 > $O/r03_01_conv1x1.log 2>&1 || { tail -30 $O/r03_01_conv1x1.log; exit 1; }
tail -3 $O/r03_01_conv1x1.log
timeout -k 10 300 python -u bench/gemm1x1.py > $O/r03_01_gemm1x1.log 2>&1 || { tail -30 $O/r03_01_gemm1x1.log; exit 1; }
cat $O/r03_01_gemm1x1.log
timeout -k 10 600 python -u bench.py > $O/r03_01_bench.log 2>&1 || { tail -20 $O/r03_01_bench.log; exit 1; }
grep '^{' $O/r03_01_bench.log | cut -c1-600
