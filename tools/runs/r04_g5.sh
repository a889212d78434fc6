#!/bin/bash
# GPU pass: gemm.hip tests, BERT batched-8 and per-rank V=1 steps, kernel profile of the batched step
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_06}; mkdir -p $O
cd $R
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_ffn_gpu.py tests/test_batched_workers_gpu.py tests/test_transformer_ops_gpu.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 --json-out $O/bert.jsonl > $O/bert.log 2>&1 || exit 1
timeout -k 10 300 python bench/configs.py --config bert_geomed --virtual-workers 1 --batch 32 --steps 20 --warmup 3 --json-out $O/bert.jsonl >> $O/bert.log 2>&1 || exit 1
timeout -k 10 300 python bench/configs.py --config bert_geomed --virtual-workers 1 --batch 64 --steps 20 --warmup 3 --json-out $O/bert.jsonl >> $O/bert.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 6 --warmup 3 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 60 --out $O/bert_kernels.md
rm -rf $O/raw
