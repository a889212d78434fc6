#!/bin/bash
# r05 pass 10: BERT linear weight gradients (wgrad1x1 vs hipBLASLt TN vs transposed NT); BERT
# configs (per-rank V = 1 x 64, batched 8 x 32) on the current code.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_10; mkdir -p $O
cd $R
timeout -k 10 300 python bench/linear_wgrad.py > $O/linear_wgrad.jsonl 2> $O/linear_wgrad.err || { tail -20 $O/linear_wgrad.err; exit 1; }
cat $O/linear_wgrad.jsonl
timeout -k 10 300 python bench/configs.py --config bert_geomed --batch 64 --steps 20 --warmup 5 --no-baseline --json-out $O/bert_v1.jsonl > $O/bert_v1.log 2>&1 || { tail -20 $O/bert_v1.log; exit 1; }
timeout -k 10 300 python bench/configs.py --config bert_geomed --batch 32 --virtual-workers 8 --steps 20 --warmup 5 --no-baseline --json-out $O/bert_v8.jsonl > $O/bert_v8.log 2>&1 || { tail -20 $O/bert_v8.log; exit 1; }
python3 -c "
import json
for f in ('bert_v1', 'bert_v8'):
    r=json.loads(open('$O/%s.jsonl' % f).readline()); print(f, r['ms_per_step'], r['tokens_per_s'], r['phase_ms_per_step'])"
