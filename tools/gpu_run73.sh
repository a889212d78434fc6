#!/bin/bash
# GPU pass 73: stem weight gradient with two LDS stages: tests, kernel timing, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_stem_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest73.log 2>&1; rc=$?
tail -2 gpurun_out/pytest73.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/diag/stem_bench.py 512 || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-baseline --json-out gpurun_out/bench73_$i.json > gpurun_out/bench73_$i.log 2>&1 || exit $?
  echo "run$i $(tail -1 gpurun_out/bench73_$i.log | cut -c90-160)"
done
