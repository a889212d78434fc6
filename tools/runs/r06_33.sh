#!/bin/bash
# r06 pass 33: gemm.hip group height 4 vs 8 (CML_GEMM_GM) on the ResNet headline and the Llama step.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_33; mkdir -p $O
cd $R
for gm in 4 8 4 8; do
  CML_GEMM_GM=$gm timeout -k 10 500 python -u bench.py --steps 10 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/b_$gm.json 2> $O/b_$gm.err || { tail -20 $O/b_$gm.err; exit 1; }
  python3 -c "
import json
r=json.loads([l for l in open('$O/b_$gm.json') if l.startswith('{')][0])
print('resnet gm $gm', r['value'], r['ms_per_step'])"
done
for gm in 4 8 4 8; do
  rm -f $O/llama_$gm.jsonl
  CML_GEMM_GM=$gm timeout -k 10 600 python -u bench/configs.py --config llama_gossip --loopback --steps 4 --warmup 2 --no-baseline --json-out $O/llama_$gm.jsonl > $O/llama_$gm.log 2>&1 || { tail -30 $O/llama_$gm.log; exit 1; }
  python3 -c "import json; r=json.loads(open('$O/llama_$gm.jsonl').readline()); print('llama gm $gm', r['ms_per_step'])"
done
