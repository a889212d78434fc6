#!/bin/bash
# Round 3, GPU pass 32: kernel profiles of the batch-2048 and batch-256 steps with the stride-2 3x3
# convs on conv_gemm.hip (rocprofv3 class tables), small-launch attribution at batch 256, batch-256
# A/B of the small-M conv_gemm tiles (128 x 128 when the 256 x 256 grid has < 512 tiles).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r03_32_* $O/raw32*
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv3x3_s2_gpu.py tests/test_bwd_fusion_gpu.py tests/test_conv1x1_bn_gpu.py > $O/r03_32_tests.txt 2>&1 || { tail -40 $O/r03_32_tests.txt; exit 1; }
tail -2 $O/r03_32_tests.txt
timeout -k 10 200 python -u bench/conv3x3_s2.py --batch 256 > $O/r03_32_shapes.jsonl 2>&1 || { tail -20 $O/r03_32_shapes.jsonl; exit 1; }
grep '^{' $O/r03_32_shapes.jsonl
timeout -k 10 300 python -u tools/small_kernels.py --batch 256 --top 60 > $O/r03_32_small256.txt 2>&1 || { tail -30 $O/r03_32_small256.txt; exit 1; }
head -5 $O/r03_32_small256.txt
for rep in 1 2; do
  for arm in default nosmallm; do
    case $arm in
      default) envs="";;
      nosmallm) envs="CML_CONV_GEMM_SMALLM=0";;
      nos2) envs="CML_CONV3X3_S2=0";;
    esac
    env $envs timeout -k 10 300 python -u bench.py --batch 256 --steps 30 --warmup 5 --no-baseline --virtual-workers 0 --b256-batch 0 > $O/r03_32_b256_$arm$rep.log 2>&1 || { tail -20 $O/r03_32_b256_$arm$rep.log; exit 1; }
    echo "b256 $arm $rep $(grep -o '"ms_per_step": [0-9.]*' $O/r03_32_b256_$arm$rep.log | head -1)" | tee -a $O/r03_32_ab.txt
  done
done
cd /tmp && export TMPDIR=/tmp
for B in 2048 256; do
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw32_$B -o run -- python3 $R/bench.py --batch $B --steps 6 --warmup 2 --no-baseline --virtual-workers 0 --b256-batch 0 --profile-marker > $O/r03_32_prof$B.log 2>&1 || { tail -20 $O/r03_32_prof$B.log; exit 1; }
db=$(find $O/raw32_$B -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 100 --out $O/r03_32_kernels_b$B.md
rm -rf $O/raw32_$B
python3 $R/tools/kernel_classes.py $O/r03_32_kernels_b$B.md | tee $O/r03_32_classes_b$B.md
done
