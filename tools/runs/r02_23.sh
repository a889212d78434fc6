#!/bin/bash
# Round 2, GPU pass 23: glds double-buffered implicit-GEMM conv vs MIOpen / TAP kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
timeout -k 10 400 python -u bench/conv3x3.py > $O/r02_23_conv3x3.jsonl 2>$O/r02_23.err || { tail -20 $O/r02_23.err; exit 1; }
cat $O/r02_23_conv3x3.jsonl
