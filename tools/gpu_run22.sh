#!/bin/bash
# GPU pass 22: Llama-3-8B gossip per-GPU batch 2 / 4 (2048-token sequences) throughput + memory.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for b in 4 2; do
timeout -k 10 400 python bench/configs.py --config llama_gossip --batch $b --steps 4 --warmup 2 --json-out gpurun_out/configs22.jsonl > gpurun_out/configs22_llama_b$b.log 2>&1 || exit $?
tail -1 gpurun_out/configs22_llama_b$b.log | cut -c200-700
done
