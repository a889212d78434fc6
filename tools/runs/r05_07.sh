#!/bin/bash
# r05 pass 7: Llama-3-8B gossip (loopback) with bias-free linears (transposed-NT weight
# gradients) + its kernel table; BERT per-rank step kernel table (128-tile GEMMs in use?);
# headline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_07; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_transformer_ops_gpu.py tests/test_engine_gpu.py tests/test_loopback.py tests/test_gram_precision_gpu.py tests/test_flash_attn_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u bench/configs.py --config llama_gossip --loopback --steps 5 --warmup 2 --no-baseline --json-out $O/llama.jsonl > $O/llama.log 2>&1 || { tail -30 $O/llama.log; exit 1; }
python3 -c "
import json
r=json.loads(open('$O/llama.jsonl').readline()); print('llama', r['ms_per_step'], r['tokens_per_s'], r['phase_ms_per_step'], r.get('max_mem_gb'))"
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json
r=json.loads([l for l in open('$O/bench.json') if l.startswith('{')][0])
print({k: r.get(k) for k in ['value','ms_per_step','agg_overhead_vs_allreduce','engine_step_ms','b256_ms_per_step','b256_allreduce_ms_per_step','b256_agg_overhead_vs_allreduce','b256_engine_step_ms','b256_allreduce_engine_step_ms']})"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/rawb -o run -- python3 $R/bench/configs.py --config bert_geomed --batch 64 --steps 10 --warmup 3 --no-baseline --profile-marker > $O/prof_bert.log 2>&1 || { tail -20 $O/prof_bert.log; exit 1; }
db=$(find $O/rawb -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 60 --out $O/bert_v1_kernels.md
rm -rf $O/rawb
head -24 $O/bert_v1_kernels.md | cut -c1-160
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/rawl -o run -- python3 $R/bench/configs.py --config llama_gossip --loopback --steps 3 --warmup 2 --no-baseline --profile-marker > $O/prof_llama.log 2>&1 || { tail -20 $O/prof_llama.log; exit 1; }
db=$(find $O/rawl -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 3 --top 60 --out $O/llama_kernels.md
rm -rf $O/rawl
head -24 $O/llama_kernels.md | cut -c1-160
