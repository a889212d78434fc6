#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_07}; mkdir -p $O
cd $R
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_ffn_gpu.py tests/test_batched_workers_gpu.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench/gemm.py --only fc1 fc2_dgrad qkv sq8k --json-out $O/gemm.jsonl > $O/gemm.log 2>&1 || exit 1
timeout -k 10 300 python bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 --json-out $O/bert.jsonl > $O/bert.log 2>&1 || exit 1
