#!/bin/bash
# r05 pass 6: BERT per-rank step (V = 1 x 64 x 128) own 128-tile GEMMs vs hipBLASLt (A/B x 2);
# Llama GEMM shapes incl. transposed-NT weight gradients; b256 Krum / all-reduce kernel tables.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_06; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_ffn_gpu.py tests/test_batched_workers_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for g in 1 0; do
    CML_OWN_GEMM128=$g timeout -k 10 300 python bench/configs.py --config bert_geomed --batch 64 --steps 20 --warmup 5 --no-baseline --json-out $O/bert_g128_$g.jsonl > $O/bert_$g.log 2>&1 || { tail -20 $O/bert_$g.log; exit 1; }
  done
done
python3 -c "
import json
for g in (1, 0):
    for l in open('$O/bert_g128_%d.jsonl' % g):
        r=json.loads(l); print('gemm128', g, r['ms_per_step'], r['tokens_per_s'])"
timeout -k 10 300 python bench/llama_gemm.py --json-out $O/llama_gemm.jsonl > $O/llama_gemm.log 2>&1 || { tail -20 $O/llama_gemm.log; exit 1; }
grep wgrad $O/llama_gemm.jsonl
cd /tmp && export TMPDIR=/tmp
for cfg in "krum sharded" "mean allreduce"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/raw_$1 -o run -- python3 $R/bench.py --rule $1 --topology $2 --batch 256 --steps 10 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof_$1.log 2>&1 || { tail -20 $O/prof_$1.log; exit 1; }
  db=$(find $O/raw_$1 -name '*.db' -print -quit)
  python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 80 --out $O/b256_$1_kernels.md
  rm -rf $O/raw_$1
  head -4 $O/b256_$1_kernels.md
done
