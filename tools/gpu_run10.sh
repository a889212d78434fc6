#!/bin/bash
# GPU pass 10: tests, headline bench (b512), batch-1024 probe, steady-state profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu10.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu10.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --json-out gpurun_out/bench10.json > gpurun_out/bench10.log 2>&1; rc=$?
tail -1 gpurun_out/bench10.log | cut -c1-300; grep warmup gpurun_out/bench10.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --steps 10 --warmup 3 --batch 1024 --no-baseline --json-out gpurun_out/bench10_b1024.json > gpurun_out/bench10_b1024.log 2>&1; rc=$?
tail -1 gpurun_out/bench10_b1024.log | cut -c1-300; grep warmup gpurun_out/bench10_b1024.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof10 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --no-baseline --profile-marker > $GRAFT_REPO_ROOT/gpurun_out/prof10.log 2>&1; rc=$?
tail -1 $GRAFT_REPO_ROOT/gpurun_out/prof10.log | cut -c1-200
exit $rc
