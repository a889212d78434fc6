#!/bin/bash
# Round 4, GPU pass 38: transformer-linear weight gradients on wgrad1x1.hip vs hipBLASLt at the
# BERT-base per-rank shapes (bench/linear_wgrad.py), the GPU test of that path, and the BERT V = 1
# x 64 step with CML_OWN_LINEAR_WGRAD off / on, two alternating pairs on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_38; mkdir -p $O
cd $R
timeout -k 10 300 python -u bench/linear_wgrad.py > $O/linear_wgrad.jsonl 2> $O/linear_wgrad.err || { tail -20 $O/linear_wgrad.err; exit 1; }
cat $O/linear_wgrad.jsonl
timeout -k 10 300 python -u -m pytest tests/test_transformer_ops_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/test.txt 2>&1 || { tail -40 $O/test.txt; exit 1; }
tail -1 $O/test.txt
for i in 1 2; do
  for s in 0 1; do
    CML_OWN_LINEAR_WGRAD=$s timeout -k 10 300 python -u bench/configs.py --config bert_geomed --virtual-workers 1 --batch 64 --loopback --steps 20 --warmup 5 > $O/bert_v1_w${s}_$i.jsonl 2> $O/bert_v1_w${s}_$i.err || { tail -20 $O/bert_v1_w${s}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d.get('ms_per_step'), d.get('value'))" $O/bert_v1_w${s}_$i.jsonl $s
  done
done
