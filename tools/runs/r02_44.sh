#!/bin/bash
# Round 2, GPU pass 44: conv_gemm narrow-tile variants on the layer-1 3x3 shape.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_44_*
for v in 0 1 2 3 0; do
CML_CONV_GEMM_NARROW=$v timeout -k 10 120 python -u tools/diag/conv_gemm_narrow.py >> $O/r02_44_narrow.jsonl 2>$O/r02_44_err.log || { tail -20 $O/r02_44_err.log; exit 1; }
done
cat $O/r02_44_narrow.jsonl
