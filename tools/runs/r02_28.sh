#!/bin/bash
# Round 2, GPU pass 28: BASELINE.json transformer configs with the current code.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -f $O/r02_28_*
timeout -k 10 400 python -u bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 --json-out $O/r02_28_configs.jsonl > $O/r02_28_bert.log 2>&1 || { tail -20 $O/r02_28_bert.log; exit 1; }
timeout -k 10 600 python -u bench/configs.py --config llama_gossip --steps 5 --warmup 2 --json-out $O/r02_28_configs.jsonl > $O/r02_28_llama.log 2>&1 || { tail -20 $O/r02_28_llama.log; exit 1; }
cut -c1-600 $O/r02_28_configs.jsonl
