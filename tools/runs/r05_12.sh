#!/bin/bash
# r05 pass 12: library weight gradients vs own kernels per shape (b2048); step time with the
# wgrad1x1 "all" set vs the core set.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_12; mkdir -p $O
cd $R
timeout -k 10 300 python -u bench/wgrad_lib.py 2048 > $O/wgrad_lib.jsonl 2> $O/wgrad_lib.err || { tail -20 $O/wgrad_lib.err; exit 1; }
cat $O/wgrad_lib.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/bench_core.log 2>&1 || { tail -20 $O/bench_core.log; exit 1; }
grep '^{' $O/bench_core.log | cut -c1-200
CML_WGRAD1X1_SET=all timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/bench_all.log 2>&1 || { tail -20 $O/bench_all.log; exit 1; }
grep '^{' $O/bench_all.log | cut -c1-200
