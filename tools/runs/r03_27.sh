#!/bin/bash
# Round 3, GPU pass 27: stem gather vs two-pass dW over batch sizes (pass 26 saw a 7 % relative
# difference at batch 2048 with the tests green at batch <= 5).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_27_*
timeout -k 10 400 python -u tools/diag/stem_gather_diag.py > $O/r03_27_diag.jsonl 2>&1 || { tail -30 $O/r03_27_diag.jsonl; exit 1; }
grep '^{' $O/r03_27_diag.jsonl
