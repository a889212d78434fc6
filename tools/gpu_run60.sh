#!/bin/bash
# GPU pass 60: own 1x1 weight gradient: tests, per-shape timing vs MIOpen, bench A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_wgrad1x1_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest60.log 2>&1; rc=$?
tail -3 gpurun_out/pytest60.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/diag/wgrad1x1_bench.py 1024 > gpurun_out/wgrad60.log || exit $?; grep own gpurun_out/wgrad60.log
for f in 1 0 1; do
  CML_WGRAD1X1=$f timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-baseline --json-out gpurun_out/bench60_w$f.json > gpurun_out/bench60_w$f.log 2>&1 || exit $?
  echo "wgrad1x1=$f $(tail -1 gpurun_out/bench60_w$f.log | cut -c90-190)"
done
