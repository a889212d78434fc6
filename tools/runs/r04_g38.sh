#!/bin/bash
# Round 4, GPU pass 38: transformer-linear weight gradients on wgrad1x1.hip vs hipBLASLt at the
# BERT-base per-rank shapes (bench/linear_wgrad.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_38; mkdir -p $O
cd $R
timeout -k 10 300 python -u bench/linear_wgrad.py > $O/linear_wgrad.jsonl 2> $O/linear_wgrad.err || { tail -20 $O/linear_wgrad.err; exit 1; }
cat $O/linear_wgrad.jsonl
