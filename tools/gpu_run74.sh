#!/bin/bash
# GPU pass 74: refresh the other BASELINE configurations with the current kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/configs74.jsonl
timeout -k 10 300 python bench/configs.py --config resnet_mkrum --virtual-workers 4 --batch 512 --steps 10 --warmup 3 --json-out $O > gpurun_out/configs74_mkrum.log 2>&1 || exit $?
tail -1 gpurun_out/configs74_mkrum.log | cut -c1-300
timeout -k 10 300 python bench/configs.py --config resnet_trimmed --virtual-workers 4 --batch 512 --steps 10 --warmup 3 --json-out $O > gpurun_out/configs74_trimmed.log 2>&1 || exit $?
tail -1 gpurun_out/configs74_trimmed.log | cut -c1-300
timeout -k 10 300 python bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 --json-out $O > gpurun_out/configs74_bert.log 2>&1 || exit $?
tail -1 gpurun_out/configs74_bert.log | cut -c1-300
timeout -k 10 500 python bench/configs.py --config llama_gossip --steps 4 --warmup 2 --json-out $O > gpurun_out/configs74_llama.log 2>&1 || exit $?
tail -1 gpurun_out/configs74_llama.log | cut -c1-300
