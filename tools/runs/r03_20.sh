#!/bin/bash
# Round 3, GPU pass 20: small-launch attribution with enclosing-op call sites (batch 256 ResNet-50).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_20_*
timeout -k 10 300 python -u tools/small_kernels.py --batch 256 --top 90 > $O/r03_20_small_b256.txt 2>&1 || { tail -30 $O/r03_20_small_b256.txt; exit 1; }
grep -v "^\[W\|Warning\|warn" $O/r03_20_small_b256.txt | head -95 | cut -c1-200
