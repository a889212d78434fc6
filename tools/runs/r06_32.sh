#!/bin/bash
# r06 pass 32: gemm.hip group height (CML_GEMM_GM 4 / 8 / 16) on the Llama-3-8B GEMM shapes.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_32; mkdir -p $O
cd $R
for gm in 8 4 16 8 4 16; do
  rm -f $O/lg_$gm.jsonl
  CML_GEMM_GM=$gm timeout -k 10 300 python -u bench/llama_gemm.py --reps 10 --json-out $O/lg_$gm.jsonl > $O/lg_$gm.log 2>&1 || { tail -20 $O/lg_$gm.log; exit 1; }
  python3 -c "
import json
for l in open('$O/lg_$gm.jsonl'):
    r=json.loads(l)
    print('gm $gm', r['shape'], r['op'], r.get('own_ms'), r.get('own_nt_ms'), r.get('blas_ms'), r.get('blas_nt_ms'))"
done
