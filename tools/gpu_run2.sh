#!/bin/bash
# GPU pass 2: kernel tests + 1-GPU bench + rocprofv3 kernel stats of the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench1.log 2>&1; rc=$?
tail -3 gpurun_out/bench1.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1; rc=$?
tail -3 $GRAFT_REPO_ROOT/gpurun_out/prof1.log
exit $rc
