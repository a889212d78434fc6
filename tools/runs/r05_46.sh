#!/bin/bash
# r05 pass 46: register-only bf16 transpose (no LDS, 8 loads in flight per lane) vs the LDS kernel:
# tests, transpose bench, Llama-3-8B step.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_46; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_transformer_ops_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python -u bench/transpose.py > $O/transpose_reg.jsonl 2> $O/t.err || { tail -20 $O/t.err; exit 1; }
CML_TRANSPOSE_LDS=1 timeout -k 10 300 python -u bench/transpose.py > $O/transpose_lds.jsonl 2> $O/t.err || { tail -20 $O/t.err; exit 1; }
cat $O/transpose_reg.jsonl $O/transpose_lds.jsonl
for k in 0 1; do
CML_TRANSPOSE_LDS=$k timeout -k 10 600 python -u bench/configs.py --config llama_gossip --loopback --steps 5 --warmup 2 --no-baseline --json-out $O/llama_lds$k.jsonl > $O/llama_lds$k.log 2>&1 || { tail -30 $O/llama_lds$k.log; exit 1; }
python3 -c "import json; r=json.loads(open('$O/llama_lds$k.jsonl').readline()); print('llama lds=$k', r['ms_per_step'], r['tokens_per_s'])"
done
