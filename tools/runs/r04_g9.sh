#!/bin/bash
# Round 4, GPU pass 9: gemm.hip with B as [K][N] (no weight transposes), padded MLM logits with the
# bias gradient from the CE backward, fused head linear + GELU: tests, BERT 8 x 32 and V = 1 steps,
# BERT kernel profile, ResNet-50 step.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_09}; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gemm_gpu.py tests/test_head_fusion_gpu.py tests/test_conv_mm_gpu.py tests/test_transformer_ops_gpu.py tests/test_batched_workers_gpu.py tests/test_ffn_gpu.py tests/test_engine_gpu.py tests/test_conv1x1g_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 --json-out $O/bert.jsonl > $O/bert.log 2>&1 || { tail -30 $O/bert.log; exit 1; }
timeout -k 10 300 python -u bench/configs.py --config bert_geomed --virtual-workers 1 --batch 32 --steps 20 --warmup 3 --json-out $O/bert.jsonl >> $O/bert.log 2>&1 || { tail -30 $O/bert.log; exit 1; }
timeout -k 10 300 python -u bench/configs.py --config bert_geomed --virtual-workers 1 --batch 64 --steps 20 --warmup 3 --json-out $O/bert.jsonl >> $O/bert.log 2>&1 || { tail -30 $O/bert.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 12 --warmup 4 --no-baseline --b256-batch 0 --virtual-workers 0 --json-out $O/resnet.json > $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 6 --warmup 3 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 60 --out $O/bert_kernels.md
rm -rf $O/raw
