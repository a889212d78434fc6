#!/bin/bash
# Round 2, GPU pass 43: stride-2 kernels per shape (bench/stride2.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_43_*
timeout -k 10 300 python -u bench/stride2.py --json-out $O/r02_43_stride2.jsonl > $O/r02_43_bench.log 2>&1 || { tail -20 $O/r02_43_bench.log; exit 1; }
cat $O/r02_43_bench.log
