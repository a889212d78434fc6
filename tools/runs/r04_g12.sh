#!/bin/bash
# Round 4, GPU pass 12: Llama-3-8B gossip config (exp graph, 1-rank RCCL loopback exchange):
# step + kernel profile of the current code.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_12}; mkdir -p $O
cd $R
timeout -k 10 600 python -u bench/configs.py --config llama_gossip --loopback --steps 5 --warmup 2 --json-out $O/llama.jsonl > $O/llama.log 2>&1 || { tail -30 $O/llama.log; exit 1; }
cut -c1-400 $O/llama.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench/configs.py --config llama_gossip --loopback --steps 3 --warmup 2 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 3 --top 60 --out $O/llama_kernels.md
rm -rf $O/raw
head -30 $O/llama_kernels.md | cut -c1-200
