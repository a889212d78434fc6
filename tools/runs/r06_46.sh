#!/bin/bash
# r06 pass 46: + one-pass avg-pool backward, bf16 stem outputs; tests, b256 A/B, kernel table.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_46; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_fin_affine_gpu.py tests/test_bwd_fusion_gpu.py tests/test_conv3x3_s2_gpu.py \
  tests/test_conv1x1_bn_gpu.py tests/test_conv1x1g_gpu.py tests/test_conv_gemm2_gpu.py \
  tests/test_conv3x3p_gpu.py tests/test_bn_gpu.py tests/test_conv3x3_layouts_gpu.py tests/test_stem_gpu.py tests/test_convergence_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for f in 1 0; do
    CML_FIN_AFFINE=$f CML_FIN_DGAMMA=$f CML_BATCH_WLAYOUTS=$f timeout -k 10 300 python3 bench.py --batch 256 --steps 40 --warmup 8 \
      --no-baseline --b256-batch 0 > $O/ab_${f}_$i.log 2>&1 || { tail -20 $O/ab_${f}_$i.log; exit 1; }
    echo "fin=$f run $i: $(grep '^{' $O/ab_${f}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --batch 256 --steps 10 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 400 --out $O/kernels_b256.md > /dev/null
rm -rf $O/raw
python3 $R/tools/kernel_classes.py $O/kernels_b256.md > $O/classes_b256.md
head -3 $O/kernels_b256.md
