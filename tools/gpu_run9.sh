#!/bin/bash
# GPU pass 9: tests (BN mask / dual-gradient links, maxpool), headline bench, steady-state profile,
# ResNet-50 multi-Krum with 8 virtual workers on one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu9.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu9.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --json-out gpurun_out/bench9.json > gpurun_out/bench9.log 2>&1; rc=$?
tail -1 gpurun_out/bench9.log; grep warmup gpurun_out/bench9.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof9 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --no-baseline --profile-marker > $GRAFT_REPO_ROOT/gpurun_out/prof9.log 2>&1; rc=$?
tail -1 $GRAFT_REPO_ROOT/gpurun_out/prof9.log
[ $rc -eq 0 ] || exit $rc
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench/conv_shapes.py --batch 512 --json-out gpurun_out/conv_shapes9.jsonl > gpurun_out/conv9.log 2>&1; rc=$?
tail -2 gpurun_out/conv9.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/configs.py --config resnet_mkrum --virtual-workers 8 --batch 64 --steps 10 --warmup 3 --json-out gpurun_out/configs9.jsonl > gpurun_out/cfg9_mkrum.log 2>&1; rc=$?
tail -1 gpurun_out/cfg9_mkrum.log
exit $rc
