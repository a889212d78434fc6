#!/bin/bash
# r06 pass 39: 3x3 conv mode vs plain GEMM at the layer-2/3/4 shapes (batch 2560).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_39; mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/diag/conv_mode_vs_gemm.py > $O/conv_mode.jsonl 2> $O/conv_mode.err || { tail -20 $O/conv_mode.err; exit 1; }
cat $O/conv_mode.jsonl
