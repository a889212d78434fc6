#!/bin/bash
# Round 4, GPU pass 24: the round's 3x3 kernels on vs off on one box (CML_CONV3P=0
# CML_CONV_GEMM2=0 = the round-start 3x3 path), three alternating pairs at batch 2048; the five
# per-config benches (1 GPU, RCCL loopback where the config exchanges).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_24}; mkdir -p $O
cd $R
B="--steps 12 --warmup 4 --no-baseline --b256-batch 0 --virtual-workers 0"
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py $B --json-out $O/resnet_new_$i.json >> $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
  CML_CONV3P=0 CML_CONV_GEMM2=0 timeout -k 10 300 python -u bench.py $B --json-out $O/resnet_old_$i.json >> $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
done
for f in $O/resnet_*.json; do python3 -c "import json,sys; print(sys.argv[1], json.load(open(sys.argv[1]))['ms_per_step'])" $f; done
for c in mlp_median resnet_trimmed resnet_mkrum bert_geomed; do
  timeout -k 10 400 python -u bench/configs.py --config $c --loopback --steps 10 --warmup 3 --json-out $O/configs.jsonl >> $O/configs.log 2>&1 || { tail -30 $O/configs.log; exit 1; }
done
timeout -k 10 600 python -u bench/configs.py --config llama_gossip --loopback --steps 5 --warmup 2 --json-out $O/configs.jsonl >> $O/configs.log 2>&1 || { tail -30 $O/configs.log; exit 1; }
python3 -c "
import json
for l in open('$O/configs.jsonl'):
    d = json.loads(l)
    print(d['config'], d.get('workers'), d.get('per_worker_batch'), d.get('ms_per_step'), d.get('samples_per_s'), d.get('tokens_per_s'))
"
