#!/bin/bash
# r05 pass 44: current numbers of the other BASELINE configs (Llama-3-8B gossip, BERT V = 1 and
# the 8-virtual-worker BERT geometric median).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_44; mkdir -p $O
cd $R
timeout -k 10 600 python -u bench/configs.py --config llama_gossip --loopback --steps 5 --warmup 2 --no-baseline --json-out $O/llama.jsonl > $O/llama.log 2>&1 || { tail -30 $O/llama.log; exit 1; }
python3 -c "import json; r=json.loads(open('$O/llama.jsonl').readline()); print('llama', r['ms_per_step'], r['tokens_per_s'])"
timeout -k 10 300 python bench/configs.py --config bert_geomed --batch 64 --steps 20 --warmup 5 --no-baseline --json-out $O/bert_v1.jsonl > $O/bert_v1.log 2>&1 || { tail -20 $O/bert_v1.log; exit 1; }
python3 -c "import json; r=json.loads(open('$O/bert_v1.jsonl').readline()); print('bert_v1', r['ms_per_step'])"
timeout -k 10 300 python bench/configs.py --config bert_geomed --batch 32 --virtual-workers 8 --steps 20 --warmup 5 --no-baseline --json-out $O/bert_v8.jsonl > $O/bert_v8.log 2>&1 || { tail -20 $O/bert_v8.log; exit 1; }
python3 -c "import json; r=json.loads(open('$O/bert_v8.jsonl').readline()); print('bert_v8', r['ms_per_step'], r.get('workers'), r.get('per_worker_batch'))"
