#!/bin/bash
# GPU pass 19: BN / conv tests with the padded stem, headline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_bn19.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_bn19.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --json-out gpurun_out/bench19.json > gpurun_out/bench19.log 2>&1; rc=$?
tail -1 gpurun_out/bench19.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc

exit $rc
