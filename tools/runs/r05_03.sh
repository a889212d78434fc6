#!/bin/bash
# r05 pass 3: headline bench with lagged compute-stream Grams; Llama-3-8B gossip (loopback, as
# r04) on the own flash attention + its kernel profile; Llama GEMM shapes own vs hipBLASLt.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_03; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gram_precision_gpu.py tests/test_loopback.py tests/test_engine_gpu.py tests/test_ffn_gpu.py tests/test_head_fusion_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 600 python -u bench/configs.py --config llama_gossip --loopback --steps 5 --warmup 2 --no-baseline --json-out $O/llama.jsonl > $O/llama.log 2>&1 || { tail -30 $O/llama.log; exit 1; }
cut -c1-300 $O/llama.jsonl
timeout -k 10 300 python bench/llama_gemm.py --json-out $O/llama_gemm.jsonl > $O/llama_gemm.log 2>&1 || { tail -20 $O/llama_gemm.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/rawl -o run -- python3 $R/bench/configs.py --config llama_gossip --loopback --steps 3 --warmup 2 --no-baseline --profile-marker > $O/prof_llama.log 2>&1 || { tail -20 $O/prof_llama.log; exit 1; }
db=$(find $O/rawl -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 3 --top 60 --out $O/llama_kernels.md
rm -rf $O/rawl
head -30 $O/llama_kernels.md | cut -c1-200
