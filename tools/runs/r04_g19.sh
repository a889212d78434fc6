#!/bin/bash
# Round 4, GPU pass 19: conv3x3p.hip staggered form (epilogue of one wave beside its SIMD
# partner's MFMAs) vs the serial form (CML_CONV3P=2) vs the implicit GEMM (0): tests, isolated
# kernels, same-box step A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_19}; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv3x3p_gpu.py tests/test_bwd_fusion_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for v in 1 2 0 1; do
  CML_CONV3P=$v timeout -k 10 120 python -u bench/conv3x3p.py --json-out $O/p3.jsonl >> $O/p3.log 2>&1 || { tail -30 $O/p3.log; exit 1; }
done
cat $O/p3.jsonl
B="--steps 12 --warmup 4 --no-baseline --b256-batch 0 --virtual-workers 0"
i=0
for v in 1 2 1 2; do
  i=$((i+1))
  CML_CONV3P=$v timeout -k 10 300 python -u bench.py $B --json-out $O/resnet_p3_${v}_$i.json >> $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
done
for f in $O/resnet_p3_*.json; do python3 -c "import json,sys; print(sys.argv[1], json.load(open(sys.argv[1]))['ms_per_step'])" $f; done
