#!/bin/bash
# GPU pass 75: stem pool forward on 2 x 2 output blocks: tests, kernel A/B, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_stem_gpu.py tests/test_bn_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest75.log 2>&1; rc=$?
tail -2 gpurun_out/pytest75.log; [ $rc -eq 0 ] || exit $rc
for b in 1 0 1 0; do echo "blocks=$b $(CML_POOL_BLOCKS=$b timeout -k 10 120 python tools/diag/stem_bench.py 1024)" || exit 1; done
for b in 1 0; do
  CML_POOL_BLOCKS=$b timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-baseline --json-out gpurun_out/bench75_p$b.json > gpurun_out/bench75_p$b.log 2>&1 || exit $?
  echo "pool_blocks=$b $(tail -1 gpurun_out/bench75_p$b.log | cut -c90-160)"
done
