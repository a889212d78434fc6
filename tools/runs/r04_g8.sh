#!/bin/bash
# Round 4, GPU pass 8: 1x1-conv GEMMs on gemm.hip (conv_mm) and the transposed-read attention
# kernels: tests, then same-box A/Bs (ResNet-50 batch 2048 step; BERT-base 8 x 32 step).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_08}; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv_mm_gpu.py tests/test_transformer_ops_gpu.py tests/test_bn_gpu.py tests/test_batched_workers_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="--steps 12 --warmup 4 --no-baseline --b256-batch 0 --virtual-workers 0"
i=0
for v in 1 0 1 0; do
  i=$((i+1))
  CML_OWN_GEMM_CONV1X1=$v timeout -k 10 300 python -u bench.py $B --json-out $O/resnet_own${v}_$i.json >> $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
done
for v in 0 1 0 1; do
  i=$((i+1))
  CML_ATTN_BWD_V1=$v timeout -k 10 300 python -u bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 --json-out $O/bert_v1_${v}_$i.jsonl >> $O/bert.log 2>&1 || { tail -30 $O/bert.log; exit 1; }
done
