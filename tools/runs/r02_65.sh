#!/bin/bash
# Round 2, GPU pass 65: attribute the remaining fill / SetTensor kernels to their ATen callers.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_65_*
timeout -k 10 300 python -u tools/torch_prof_fills.py --batch 512 > $O/r02_65_fills.txt 2>&1 || { tail -30 $O/r02_65_fills.txt; exit 1; }
tail -60 $O/r02_65_fills.txt | cut -c1-250
