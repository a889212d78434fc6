#!/bin/bash
# GPU pass 3: all GPU tests + bench + rocprof stats (fused BN kernels).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench3.log 2>&1; rc=$?
tail -2 gpurun_out/bench3.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof3.log 2>&1; rc=$?
tail -2 $GRAFT_REPO_ROOT/gpurun_out/prof3.log
exit $rc
