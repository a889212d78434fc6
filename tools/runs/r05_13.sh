#!/bin/bash
# r05 pass 13: LDS-DMA wgrad1x1 variant: tests, per-shape bench (DMA on / off), step time with
# the core / wide own-wgrad sets.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_13; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad1x1_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
timeout -k 10 300 python -u bench/wgrad_lib.py 2048 > $O/wgrad_lib_dma.jsonl 2> $O/wgrad_lib.err || { tail -20 $O/wgrad_lib.err; exit 1; }
cat $O/wgrad_lib_dma.jsonl
CML_WGRAD_DMA=0 timeout -k 10 300 python -u bench/wgrad_lib.py 2048 > $O/wgrad_lib_nodma.jsonl 2>> $O/wgrad_lib.err || { tail -20 $O/wgrad_lib.err; exit 1; }
cat $O/wgrad_lib_nodma.jsonl
for set in core wide; do
CML_WGRAD1X1_SET=$set timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/bench_$set.log 2>&1 || { tail -20 $O/bench_$set.log; exit 1; }
grep '^{' $O/bench_$set.log | cut -c1-200
done
