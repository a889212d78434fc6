#!/bin/bash
# Round 4, GPU pass 14: the patch-resident layer-1 3x3 conv (conv3x3p.hip, CML_CONV3P): its tests
# and the conv / backward-fusion suites that route through it, same-box step A/Bs at batch 2048,
# kernel table of the default step.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_14}; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv3x3p_gpu.py > $O/pytest_p3.log 2>&1 || { tail -40 $O/pytest_p3.log; exit 1; }
tail -2 $O/pytest_p3.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread -p no:cacheprovider tests/test_bwd_fusion_gpu.py tests/test_conv_gemm2_gpu.py tests/test_conv3x3_layouts_gpu.py tests/test_conv3x3_s2_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="--steps 12 --warmup 4 --no-baseline --b256-batch 0 --virtual-workers 0"
i=0
for v in 1 0 1 0; do
  i=$((i+1))
  CML_CONV3P=$v timeout -k 10 300 python -u bench.py $B --json-out $O/resnet_p3_${v}_$i.json >> $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
done
grep -h '"ms_per_step"' $O/resnet_p3_*.json | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step']) for l in sys.stdin]" || true
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --steps 6 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 400 --out $O/kernels_b2048.md
python3 $R/tools/kernel_classes.py $O/kernels_b2048.md > $O/classes_b2048.md || true
rm -rf $O/raw
grep -i "conv3x3p\|conv_gemm_kernel<256, 64" $O/kernels_b2048.md | cut -c1-220
cat $O/classes_b2048.md
