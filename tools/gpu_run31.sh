#!/bin/bash
# GPU pass 31: PyTorch TunableOp (hipBLASLt + rocBLAS solution search) for every GEMM of the
# ResNet-50 step: tune on the 1x1-conv GEMM shapes (bench/conv_shapes.py, also re-measuring GEMM
# vs MIOpen with tuned GEMMs), then the full bench step (remaining shapes), then a tuned-only
# bench run. Results file -> gpurun_out/tunableop/.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/tunableop
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1
export PYTORCH_TUNABLEOP_FILENAME=$R/gpurun_out/tunableop/resnet50_b512_%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=8 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=10
timeout -k 10 700 python -u bench/conv_shapes.py --reps 5 --json-out gpurun_out/conv_shapes31.jsonl > gpurun_out/conv_shapes31.log 2>&1; rc=$?
tail -2 gpurun_out/conv_shapes31.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --no-baseline > gpurun_out/bench31_tune.log 2>&1; rc=$?
tail -1 gpurun_out/bench31_tune.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
wc -l gpurun_out/tunableop/*
export PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_VERBOSE=0
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --json-out gpurun_out/bench31_tuned.json > gpurun_out/bench31_tuned.log 2>&1; rc=$?
tail -1 gpurun_out/bench31_tuned.log | cut -c1-200
exit $rc
