#!/bin/bash
# Round 2, GPU pass 15: per-stage A/B of the identity-tail backward fusion.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
timeout -k 10 500 python -u bench/bwd_fusion.py > $O/r02_15_bwdfusion.jsonl 2>$O/r02_15.err || { tail -20 $O/r02_15.err; exit 1; }
cat $O/r02_15_bwdfusion.jsonl
