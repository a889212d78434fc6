#!/bin/bash
# Round 4, GPU pass 23 (co tile 128, precomputed DMA slots, partial last chunks): stride-2 3x3 weight gradient on wgrad3x3s2.hip: tests, isolated kernel vs
# MIOpen at the ResNet-50 shapes (batch 2048), same-box step A/B (CML_WGRAD3X3_S2).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_23}; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_wgrad3x3s2_gpu.py tests/test_conv3x3_s2_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
timeout -k 10 300 python -u bench/wgrad3x3s2.py --json-out $O/w2.jsonl > $O/w2.log 2>&1 || { tail -30 $O/w2.log; exit 1; }
cat $O/w2.jsonl
B="--steps 12 --warmup 4 --no-baseline --b256-batch 0 --virtual-workers 0"
i=0
for v in 1 0 1 0; do
  i=$((i+1))
  CML_WGRAD3X3_S2=$v timeout -k 10 300 python -u bench.py $B --json-out $O/resnet_ws2_${v}_$i.json >> $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
done
for f in $O/resnet_ws2_*.json; do python3 -c "import json,sys; print(sys.argv[1], json.load(open(sys.argv[1]))['ms_per_step'])" $f; done
