#!/bin/bash
# GPU pass 26: gossip per-bucket optimizer update during backward (tests, Llama-3-8B batch 4 / 1
# with and without), norm backward with the residual gradient prefetched (transformer tests, BERT).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_transformer_ops_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest26.log 2>&1; rc=$?
tail -3 gpurun_out/pytest26.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench/configs.py --config llama_gossip --steps 4 --warmup 2 --json-out gpurun_out/configs26.jsonl > gpurun_out/configs26_llama.log 2>&1; rc=$?
tail -1 gpurun_out/configs26_llama.log | cut -c200-600
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench/configs.py --config llama_gossip --batch 1 --steps 5 --warmup 2 --json-out gpurun_out/configs26.jsonl > gpurun_out/configs26_llama_b1.log 2>&1; rc=$?
tail -1 gpurun_out/configs26_llama_b1.log | cut -c200-600
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 --json-out gpurun_out/configs26.jsonl > gpurun_out/configs26_bert.log 2>&1; rc=$?
tail -1 gpurun_out/configs26_bert.log | cut -c200-600
exit $rc
