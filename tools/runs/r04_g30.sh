#!/bin/bash
# Round 4, GPU pass 30: kernel profile of the BERT per-rank step (V = 1, 64 x 128 tokens).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_30}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench/configs.py --config bert_geomed --virtual-workers 1 --batch 64 --loopback --steps 10 --warmup 3 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 60 --out $O/bert_v1_kernels.md
rm -rf $O/raw
head -45 $O/bert_v1_kernels.md | cut -c1-200
