#!/bin/bash
# GPU pass 34: tree split-search and lasso kernel tests and the reference-timing rows (RF / lasso).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_select_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest34.log 2>&1; rc=$?
tail -15 gpurun_out/pytest34.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/reference_timings.py > gpurun_out/reftime34.log 2>&1; rc=$?
tail -6 gpurun_out/reftime34.log | cut -c1-250
exit $rc
