#!/bin/bash
# Round 4, GPU pass 11: stride-1 3x3 convs on gemm.hip's schedule and side-stream weight
# gradients -- tests, same-box step A/Bs at batch 2048 (CML_CONV_GEMM2, CML_SIDE_WGRAD) and batch
# 256 (CML_SIDE_WGRAD), kernel table of the default step; the batch-2048 fused-vs-library
# convergence check (noise 6) with a heartbeat file while MIOpen compiles.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_11}; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread -p no:cacheprovider tests/test_side_wgrad_gpu.py tests/test_conv1x1_bn_gpu.py tests/test_bwd_fusion_gpu.py tests/test_conv3x3_s2_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
CML_CONV_GEMM2=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread -p no:cacheprovider tests/test_conv_gemm2_gpu.py tests/test_conv1x1_bn_gpu.py tests/test_bwd_fusion_gpu.py > $O/pytest_g2.log 2>&1 || { tail -40 $O/pytest_g2.log; exit 1; }
tail -2 $O/pytest_g2.log
B="--steps 12 --warmup 4 --no-baseline --b256-batch 0 --virtual-workers 0"
i=0
for v in "1 0" "0 0" "1 1" "1 0" "0 0" "1 1"; do
  set -- $v
  i=$((i+1))
  CML_CONV_GEMM2=$1 CML_SIDE_WGRAD=$2 timeout -k 10 300 python -u bench.py $B --json-out $O/resnet_g2_$1_side_$2_$i.json >> $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
done
for s in 0 1 0 1; do
  i=$((i+1))
  CML_SIDE_WGRAD=$s timeout -k 10 300 python -u bench.py --batch 256 --steps 30 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 --json-out $O/b256_side_${s}_$i.json >> $O/resnet.log 2>&1 || { tail -30 $O/resnet.log; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --steps 6 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 400 --out $O/kernels_b2048.md
python3 $R/tools/kernel_classes.py $O/kernels_b2048.md > $O/classes_b2048.md || true
rm -rf $O/raw
cd $R
( while sleep 50; do date >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 900 python -u bench/convergence.py --steps 30 --batch 2048 --no-krum --noise 6 --noise-floor 0.004 --out $O/conv2048 > $O/conv2048.log 2>&1
rc=$?
kill $HB
[ $rc -eq 0 ] || { tail -30 $O/conv2048.log; exit 1; }
tail -1 $O/conv2048.log | cut -c1-1500
