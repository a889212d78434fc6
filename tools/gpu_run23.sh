#!/bin/bash
# GPU pass 23: BN kernels with 2-4 rows in flight per lane: tests, bench, steady profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_bn23.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_bn23.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --json-out gpurun_out/bench23.json > gpurun_out/bench23.log 2>&1; rc=$?
tail -1 gpurun_out/bench23.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/raw23 -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-baseline --profile-marker > $R/gpurun_out/prof23.log 2>&1 || exit $?
db=$(find $R/gpurun_out/raw23 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 45 --out $R/gpurun_out/prof23_resnet_kernels.md
rm -rf $R/gpurun_out/raw23
