#!/bin/bash
# GPU pass 18: BN / conv tests (finalize fold geometry, downsample link tap), headline bench,
# stem padding micro-bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_bn18.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_bn18.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --json-out gpurun_out/bench18.json > gpurun_out/bench18.log 2>&1; rc=$?
tail -1 gpurun_out/bench18.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/stem_pad.py > gpurun_out/stem_pad18.jsonl 2> gpurun_out/stem_pad18.log; rc=$?
cat gpurun_out/stem_pad18.jsonl
exit $rc
