#!/bin/bash
# r05 pass 27: direct gradients (TopologyConfig.direct_grads): tests; Llama and BERT V = 1 steps
# with / without.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_27; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_direct_grads_gpu.py tests/test_batched_workers_gpu.py tests/test_transformer_ops_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for d in 1 0; do
timeout -k 10 600 python -u bench/configs.py $( [ $d = 0 ] && echo --no-direct-grads ) --config llama_gossip --loopback --steps 5 --warmup 2 --no-baseline --json-out $O/llama_d$d.jsonl > $O/llama_d$d.log 2>&1 || { tail -30 $O/llama_d$d.log; exit 1; }
python3 -c "import json
r=json.loads(open('$O/llama_d$d.jsonl').readline()); print('llama direct=$d', r['ms_per_step'], r['tokens_per_s'], r.get('max_mem_gb'))"
done
for d in 1 0 1 0; do
timeout -k 10 300 python bench/configs.py $( [ $d = 0 ] && echo --no-direct-grads ) --config bert_geomed --batch 64 --steps 20 --warmup 5 --no-baseline --json-out $O/bert_v1_d$d.jsonl > $O/bert_v1_d$d.log 2>&1 || { tail -20 $O/bert_v1_d$d.log; exit 1; }
python3 -c "import json
r=json.loads(open('$O/bert_v1_d$d.jsonl').readline()); print('bert_v1 direct=$d', r['ms_per_step'])"
done
