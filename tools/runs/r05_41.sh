#!/bin/bash
# r05 pass 41: per-shape A/B of the register-staged vs quad (LDS-DMA) fused 1x1 kernels after the
# quad loop fix (profiles/r05_32), batch 2048.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_41; mkdir -p $O
cd $R
timeout -k 10 600 python -u bench/conv1x1g.py --reps 10 --json-out $O/c1g.json > $O/c1g.log 2>&1 || { tail -20 $O/c1g.log; exit 1; }
cat $O/c1g.log | cut -c1-260
