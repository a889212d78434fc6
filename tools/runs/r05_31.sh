#!/bin/bash
# r05 pass 31: double-buffered x in the register-staged fused 1x1 kernel (CML_C1_DB): tests with
# it on, alternating step A/B, same-box kernel tables.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_31; mkdir -p $O
cd $R
CML_C1_DB=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bn_gpu.py tests/test_bwd_fusion_gpu.py tests/test_conv1x1_bn_gpu.py tests/test_conv3x3_s2_gpu.py tests/test_conv_mm_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for rep in 1 2; do
for c in 0 1; do
CML_C1_DB=$c timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/bench_${c}_${rep}.log 2>&1 || { tail -20 $O/bench_${c}_${rep}.log; exit 1; }
echo "db=$c rep=$rep $(grep '^{' $O/bench_${c}_${rep}.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
done
cd /tmp && export TMPDIR=/tmp
for c in 0 1; do
CML_C1_DB=$c timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw$c -o run -- python3 $R/bench.py --steps 6 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof$c.log 2>&1 || { tail -20 $O/prof$c.log; exit 1; }
db=$(find $O/raw$c -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 400 --out $O/kernels_db$c.md
rm -rf $O/raw$c
head -2 $O/kernels_db$c.md | tail -1
done
