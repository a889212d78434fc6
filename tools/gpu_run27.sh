#!/bin/bash
# GPU pass 27: MFMA short-sequence attention (tests, BERT config with / without, profile).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_transformer_ops_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest27.log 2>&1; rc=$?
tail -25 gpurun_out/pytest27.log
[ $rc -eq 0 ] || exit $rc
for ak in 1 0; do
CML_ATTN_KERNEL=$ak timeout -k 10 300 python bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 --json-out gpurun_out/configs27.jsonl > gpurun_out/configs27_bert_ak$ak.log 2>&1 || exit $?
echo "attn_kernel=$ak $(tail -1 gpurun_out/configs27_bert_ak$ak.log | cut -c300-430)"
done
