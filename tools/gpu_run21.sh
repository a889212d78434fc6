#!/bin/bash
# GPU pass 21: BERT config A/B of the gradient-capture copy (HIP multi-copy vs _foreach_copy_).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for mc in 1 0 1 0; do
CML_MULTI_COPY=$mc timeout -k 10 300 python bench/configs.py --config bert_geomed --virtual-workers 8 --batch 32 --steps 10 --warmup 3 > gpurun_out/configs21_bert_mc$mc.log 2>&1 || exit $?
echo "mc=$mc $(tail -1 gpurun_out/configs21_bert_mc$mc.log | cut -c300-420)"
done
