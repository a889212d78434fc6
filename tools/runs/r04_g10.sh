#!/bin/bash
# Round 4, GPU pass 10: LDS-tiled weight transposes (b_kn GEMM reverted), tests; BERT 8 x 32 / V = 1
# steps; ResNet-50 A/B of the own 1x1 weight-gradient set (core vs all); the batch-2048
# fused-vs-library convergence check with its noise floor.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_10}; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gemm_gpu.py tests/test_head_fusion_gpu.py tests/test_conv_mm_gpu.py tests/test_transformer_ops_gpu.py tests/test_batched_workers_gpu.py tests/test_ffn_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 8 8; do
  timeout -k 10 300 python -u bench/configs.py --config bert_geomed --virtual-workers $v --batch 32 --steps 10 --warmup 3 --json-out $O/bert.jsonl >> $O/bert.log 2>&1 || { tail -30 $O/bert.log; exit 1; }
done
timeout -k 10 300 python -u bench/configs.py --config bert_geomed --virtual-workers 1 --batch 32 --steps 20 --warmup 3 --json-out $O/bert.jsonl >> $O/bert.log 2>&1 || { tail -30 $O/bert.log; exit 1; }
timeout -k 10 300 python -u bench/configs.py --config bert_geomed --virtual-workers 1 --batch 64 --steps 20 --warmup 3 --json-out $O/bert.jsonl >> $O/bert.log 2>&1 || { tail -30 $O/bert.log; exit 1; }
B="--steps 12 --warmup 4 --no-baseline --b256-batch 0 --virtual-workers 0"
i=0
for s in core all core all; do
  i=$((i+1))
  CML_WGRAD1X1_SET=$s timeout -k 10 300 python -u bench.py $B --json-out $O/resnet_wg_${s}_$i.json >> $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
done
timeout -k 10 900 python -u bench/convergence.py --steps 30 --batch 2048 --no-krum --noise 2 --noise-floor 0.004 --out $O/conv2048 > $O/conv2048.log 2>&1 || { tail -30 $O/conv2048.log; exit 1; }
tail -1 $O/conv2048.log | cut -c1-1500
