#!/bin/bash
# r05 pass 34: HBM stream rates per access mix (read / write / copy / 2:1).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_34; mkdir -p $O
cd $R
timeout -k 10 300 python -u bench/hbm_rates.py > $O/hbm.jsonl 2> $O/hbm.err || { tail -20 $O/hbm.err; exit 1; }
cat $O/hbm.jsonl
