#!/bin/bash
# r05 pass 20: two-step x prefetch in the register-staged fused 1x1 kernel (CML_C1_PF2): tests,
# alternating step A/B, kernel table.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_20; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_gpu.py tests/test_bwd_fusion_gpu.py tests/test_conv1x1_bn_gpu.py tests/test_conv1x1g_gpu.py tests/test_conv3x3_s2_gpu.py tests/test_conv_mm_gpu.py tests/test_stem_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for rep in 1 2; do
for pf in 0 1; do
CML_C1_PF2=$pf timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/bench_${pf}_${rep}.log 2>&1 || { tail -20 $O/bench_${pf}_${rep}.log; exit 1; }
echo "pf2=$pf rep=$rep $(grep '^{' $O/bench_${pf}_${rep}.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --steps 6 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 400 --out $O/kernels_b2048.md
python3 $R/tools/kernel_classes.py $O/kernels_b2048.md > $O/classes_b2048.md || true
rm -rf $O/raw
head -3 $O/kernels_b2048.md; cat $O/classes_b2048.md
