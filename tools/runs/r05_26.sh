#!/bin/bash
# r05 pass 26: multi_copy with a size-adaptive grid: test + isolated throughput.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_26; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k multi_copy > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python -u bench/multi_copy.py > $O/multi_copy.jsonl 2> $O/mc.err || { tail -20 $O/mc.err; exit 1; }
cat $O/multi_copy.jsonl
