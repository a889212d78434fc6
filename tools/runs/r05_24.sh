#!/bin/bash
# r05 pass 24: Llama-3-8B loopback gossip step with the new multi_copy: bench + kernel table.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_24; mkdir -p $O
cd $R
timeout -k 10 600 python -u bench/configs.py --config llama_gossip --loopback --steps 5 --warmup 2 --no-baseline --json-out $O/llama.jsonl > $O/llama.log 2>&1 || { tail -30 $O/llama.log; exit 1; }
python3 -c "import json
r=json.loads(open('$O/llama.jsonl').readline()); print('llama', r['ms_per_step'], r['tokens_per_s'], r['phase_ms_per_step'], r.get('max_mem_gb'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/rawl -o run -- python3 $R/bench/configs.py --config llama_gossip --loopback --steps 3 --warmup 2 --no-baseline --profile-marker > $O/prof_llama.log 2>&1 || { tail -20 $O/prof_llama.log; exit 1; }
db=$(find $O/rawl -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 3 --top 80 --out $O/llama_kernels.md
rm -rf $O/rawl
head -30 $O/llama_kernels.md | cut -c1-170
