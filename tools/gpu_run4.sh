#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench4.log 2>&1; rc=$?
tail -1 gpurun_out/bench4.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 20 --warmup 5 --miopen-find --no-baseline > gpurun_out/bench4_find.log 2>&1; rc=$?
tail -1 gpurun_out/bench4_find.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof4.log 2>&1; rc=$?
exit $rc
