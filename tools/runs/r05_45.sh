#!/bin/bash
# r05 pass 45: BN-backward apply with 4 rows in flight per thread (CML_BN_APPLY_U=4) vs 2: tests,
# kernel tables of both.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_45; mkdir -p $O
cd $R
CML_BN_APPLY_U=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bn_gpu.py tests/test_bwd_fusion_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
cd /tmp && export TMPDIR=/tmp
for u in 2 4 2 4; do
CML_BN_APPLY_U=$u timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw$u -o run -- python3 $R/bench.py --steps 6 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof$u.log 2>&1 || { tail -20 $O/prof$u.log; exit 1; }
db=$(find $O/raw$u -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 400 --out $O/kernels_u$u.md > /dev/null
rm -rf $O/raw$u
echo "U=$u $(head -2 $O/kernels_u$u.md | tail -1)"
grep -E "bn_bwd_apply_kernel<1" $O/kernels_u$u.md | cut -c1-200
done
