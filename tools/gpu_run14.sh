#!/bin/bash
# GPU pass 14: transformer-op kernel tests, then BERT-base geomed and Llama-3-8B gossip configs with
# the fused transformer kernels (compare profiles/r01_configs5.jsonl: 89.9 / 244.9 ms per step).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_transformer_ops_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_tops14.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_tops14.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 --json-out gpurun_out/configs14.jsonl > gpurun_out/configs14_bert.log 2>&1; rc=$?
tail -1 gpurun_out/configs14_bert.log | cut -c1-500
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench/configs.py --config llama_gossip --steps 5 --warmup 2 --json-out gpurun_out/configs14.jsonl > gpurun_out/configs14_llama.log 2>&1; rc=$?
tail -1 gpurun_out/configs14_llama.log | cut -c1-500
exit $rc
