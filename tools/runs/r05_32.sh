#!/bin/bash
# r05 pass 32: quad 1x1 kernel without the compiler's vmcnt(0) drains (restrict LDS helpers):
# tests, step A/B of the policies, kernel tables.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_32; mkdir -p $O
cd $R
CML_C1G=3 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv1x1g_gpu.py tests/test_bwd_fusion_gpu.py tests/test_conv1x1_bn_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
run() {   # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  echo "$tag $(grep '^{' $O/$tag.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
}
for rep in 1 2; do
run auto_$rep CML_NONE=1
run cat_$rep CML_C1G_CAT=1
run all_$rep CML_C1G=3
done
cd /tmp && export TMPDIR=/tmp
for m in 2 3; do
CML_C1G=$m timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw$m -o run -- python3 $R/bench.py --steps 6 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof$m.log 2>&1 || { tail -20 $O/prof$m.log; exit 1; }
db=$(find $O/raw$m -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 400 --out $O/kernels_c1g$m.md
rm -rf $O/raw$m
head -2 $O/kernels_c1g$m.md | tail -1
done
