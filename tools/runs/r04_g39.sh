#!/bin/bash
# Round 4, GPU pass 39 (final code): BERT V = 1 x 64 with the linear weight gradients on
# wgrad1x1.hip by default, then pass 26's full validation (GPU suite, smoke(), default bench line,
# batch-2048 kernel profile).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_39; mkdir -p $O
cd $R
timeout -k 10 300 python -u bench/configs.py --config bert_geomed --virtual-workers 1 --batch 64 --loopback --steps 20 --warmup 5 > $O/bert_v1.jsonl 2> $O/bert_v1.err || { tail -20 $O/bert_v1.err; exit 1; }
tail -1 $O/bert_v1.jsonl | cut -c1-200
OUT=r04_39 bash $R/tools/runs/r04_g26.sh
