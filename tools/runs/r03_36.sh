#!/bin/bash
# Round 3, GPU pass 36: kernel profile of the BERT-base geomed config (8 virtual workers x 32, seq 128)
# with the round-3 code: dispatches per step and the kernel table.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_36_* $O/raw36*
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw36 -o run -- python3 $R/bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 6 --warmup 3 --profile-marker > $O/r03_36_prof.log 2>&1 || { tail -20 $O/r03_36_prof.log; exit 1; }
db=$(find $O/raw36 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 60 --out $O/r03_36_bert_kernels.md
rm -rf $O/raw36
head -4 $O/r03_36_bert_kernels.md
