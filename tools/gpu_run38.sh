#!/bin/bash
# GPU pass 38: fused stem BN + ReLU + max-pool: tests, bench A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest38.log 2>&1; rc=$?
tail -15 gpurun_out/pytest38.log
[ $rc -eq 0 ] || exit $rc
for f in 1 0 1; do
CML_FUSE_STEM_POOL=$f timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-baseline --json-out gpurun_out/bench38_f$f.json > gpurun_out/bench38_f$f.log 2>&1 || exit $?
echo "fuse=$f $(tail -1 gpurun_out/bench38_f$f.log | cut -c90-170)"
done
