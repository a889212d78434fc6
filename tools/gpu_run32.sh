#!/bin/bash
# GPU pass 32: TunableOp for the BERT-base config GEMMs (tune run, then tuned run vs default).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/tunableop
timeout -k 10 300 python bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 > gpurun_out/configs32_default.log 2>&1 || exit $?
echo "default $(tail -1 gpurun_out/configs32_default.log | cut -c300-420)"
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1
export PYTORCH_TUNABLEOP_FILENAME=$R/gpurun_out/tunableop/bert_base_b32_%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=30
timeout -k 10 600 python -u bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 1 --warmup 1 > gpurun_out/configs32_tune.log 2>&1 || exit $?
wc -l gpurun_out/tunableop/bert_base_b32_0.csv
export PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_VERBOSE=0
timeout -k 10 300 python bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 > gpurun_out/configs32_tuned.log 2>&1 || exit $?
echo "tuned $(tail -1 gpurun_out/configs32_tuned.log | cut -c300-420)"
