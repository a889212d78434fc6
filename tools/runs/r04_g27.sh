#!/bin/bash
# Round 4, GPU pass 27: conv3x3p with the epilogue image accesses as asm (no compiler vmcnt(0)
# before them) and EP 2's z loaded a tile ahead; multi_copy for same-strided dense tensors. Tests,
# isolated kernels, same-box step A/B against the round-start 3x3 path.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_27}; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv3x3p_gpu.py tests/test_bwd_fusion_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for v in 1 0; do
  CML_CONV3P=$v timeout -k 10 120 python -u bench/conv3x3p.py --json-out $O/p3.jsonl >> $O/p3.log 2>&1 || { tail -30 $O/p3.log; exit 1; }
done
cat $O/p3.jsonl
B="--steps 12 --warmup 4 --no-baseline --b256-batch 0 --virtual-workers 0"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $B --json-out $O/resnet_new_$i.json >> $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
  CML_CONV3P=0 CML_CONV_GEMM2=0 timeout -k 10 300 python -u bench.py $B --json-out $O/resnet_old_$i.json >> $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
done
for f in $O/resnet_*.json; do python3 -c "import json,sys; print(sys.argv[1], json.load(open(sys.argv[1]))['ms_per_step'])" $f; done
