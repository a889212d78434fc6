#!/bin/bash
# GPU pass 20: multi-copy gradient capture (tests, Llama-3-8B gossip and BERT configs).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest20.log 2>&1; rc=$?
tail -3 gpurun_out/pytest20.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench/configs.py --config llama_gossip --steps 5 --warmup 2 --json-out gpurun_out/configs20.jsonl > gpurun_out/configs20_llama.log 2>&1; rc=$?
tail -1 gpurun_out/configs20_llama.log | cut -c1-500
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 --json-out gpurun_out/configs20.jsonl > gpurun_out/configs20_bert.log 2>&1; rc=$?
tail -1 gpurun_out/configs20_bert.log | cut -c1-500
exit $rc
