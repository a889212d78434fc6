#!/bin/bash
# GPU pass 29: BERT residual-gradient links + no materialised zero gradients: tests, config.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_transformer_ops_gpu.py tests/test_engine_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest29.log 2>&1; rc=$?
tail -3 gpurun_out/pytest29.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 --json-out gpurun_out/configs29.jsonl > gpurun_out/configs29_bert.log 2>&1 || exit $?
tail -1 gpurun_out/configs29_bert.log | cut -c200-500
timeout -k 10 300 python bench/configs.py --config bert_geomed --virtual-workers 8 --steps 10 --warmup 3 --json-out gpurun_out/configs29.jsonl > gpurun_out/configs29_bert64.log 2>&1 || exit $?
tail -1 gpurun_out/configs29_bert64.log | cut -c200-500
