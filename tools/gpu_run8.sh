#!/bin/bash
# GPU pass 8: tests; bench A/B (1x1 convs as GEMMs + residual link vs MIOpen 1x1) with naive
# solvers skipped in find; steady-state rocprof of the new default; agg micro-bench (aligned D).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu8.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu8.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --steps 20 --warmup 3 --json-out gpurun_out/bench8_gemm.json > gpurun_out/bench8_gemm.log 2>&1; rc=$?
tail -1 gpurun_out/bench8_gemm.log; grep warmup gpurun_out/bench8_gemm.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-baseline --conv1x1 miopen --json-out gpurun_out/bench8_miopen.json > gpurun_out/bench8_miopen.log 2>&1; rc=$?
tail -1 gpurun_out/bench8_miopen.log; grep warmup gpurun_out/bench8_miopen.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof8 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --no-baseline --profile-marker > $GRAFT_REPO_ROOT/gpurun_out/prof8.log 2>&1; rc=$?
tail -1 $GRAFT_REPO_ROOT/gpurun_out/prof8.log
[ $rc -eq 0 ] || exit $rc
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench/agg_kernels.py --n 4 8 16 --json-out gpurun_out/agg_kernels8.jsonl > gpurun_out/agg8.log 2>&1; rc=$?
tail -3 gpurun_out/agg8.log
exit $rc
