#!/bin/bash
# Round 2, GPU pass 18: BN apply-pass variants (rows in flight, non-temporal stores).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
timeout -k 10 400 python -u bench/bn_kernels.py --variants > $O/r02_18_bnvar.jsonl 2>$O/r02_18.err || { tail -20 $O/r02_18.err; exit 1; }
cat $O/r02_18_bnvar.jsonl
