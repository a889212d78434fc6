#!/bin/bash
# GPU pass 17: conv1x1 policy tests, headline bench with the per-shape 1x1 GEMM policy (auto) vs
# MIOpen-only, steady-state profile of the auto run.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_bn17.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_bn17.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --json-out gpurun_out/bench17_auto.json > gpurun_out/bench17_auto.log 2>&1; rc=$?
tail -1 gpurun_out/bench17_auto.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-baseline --conv1x1 miopen --json-out gpurun_out/bench17_miopen.json > gpurun_out/bench17_miopen.log 2>&1; rc=$?
tail -1 gpurun_out/bench17_miopen.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/raw17 -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-baseline --profile-marker > $R/gpurun_out/prof17.log 2>&1 || exit $?
db=$(find $R/gpurun_out/raw17 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 45 --out $R/gpurun_out/prof17_resnet_kernels.md
rm -rf $R/gpurun_out/raw17
