#!/bin/bash
# r06 pass 15: gemm.hip tile order A/B (CML_GEMM_GM 0 = n fastest, 4 / 8 = grouped m-tiles) at
# 8192^3 / 4096^3 and the Llama forward shapes, hipBLASLt alongside; GEMM tests with grouping on.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_15; mkdir -p $O
cd $R
CML_GEMM_GM=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for gm in 0 4 8 0 4; do
  CML_GEMM_GM=$gm timeout -k 10 300 python -u bench/gemm.py --only sq8k --reps 20 > $O/sq_$gm.jsonl 2> $O/sq_$gm.err || { tail -20 $O/sq_$gm.err; exit 1; }
  CML_GEMM_GM=$gm timeout -k 10 300 python -u bench/llama_gemm.py --only wqkv w13 out --reps 8 > $O/ll_$gm.jsonl 2> $O/ll_$gm.err || { tail -20 $O/ll_$gm.err; exit 1; }
  python3 - <<PY
import json
r=json.loads(open('$O/sq_$gm.jsonl').readline())
out=[('sq8k', r['own_tflops'], r['blas_tflops'])]
for l in open('$O/ll_$gm.jsonl'):
    x=json.loads(l)
    if x['op']=='fwd' and 'own_tflops' in x: out.append((x['shape'], x['own_tflops'], x['blas_tflops']))
print('gm $gm', out)
PY
done
