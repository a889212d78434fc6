#!/bin/bash
# r06 pass 16: Llama-3-8B GEMM shapes with gemm.hip's grouped tile order (default now): all three
# products of every projection, own vs hipBLASLt; BERT shapes.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_16; mkdir -p $O
cd $R
timeout -k 10 600 python -u bench/llama_gemm.py --reps 8 --json-out $O/llama_gemm.jsonl > $O/llama_gemm.log 2>&1 || { tail -20 $O/llama_gemm.log; exit 1; }
python3 - <<PY
import json
for l in open('$O/llama_gemm.jsonl'):
    x=json.loads(l)
    print(x['shape'], x['op'], {k: x[k] for k in x if k.endswith('tflops') or k=='transpose_ms'})
PY
timeout -k 10 300 python -u bench/gemm.py --json-out $O/gemm.jsonl > $O/gemm.log 2>&1 || { tail -20 $O/gemm.log; exit 1; }
python3 - <<PY
import json
for l in open('$O/gemm.jsonl'):
    x=json.loads(l)
    print(x['shape'], x.get('own_tflops'), x.get('own128_tflops'), x['blas_tflops'], x['pick'])
PY
