#!/bin/bash
# Round 4, GPU pass 17: conv3x3p.hip forward + statistics with its MFMA loop's LDS reads cut
# (weights read once per tile / patch read once per tile) -- is the loop LDS-bound?
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_17}; mkdir -p $O
cd $R
for d in 0 4 8 6 10; do
  CML_CONV3P_DBG=$d timeout -k 10 120 python -u bench/conv3x3p.py --json-out $O/p3.jsonl >> $O/p3.log 2>&1 || { tail -30 $O/p3.log; exit 1; }
done
grep fwd_stats $O/p3.jsonl
