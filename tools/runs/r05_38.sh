#!/bin/bash
# r05 pass 38: BN + residual + ReLU epilogue (SM_BNRES, MT = 2) with the residual rows loaded one
# batch ahead: tests, step, kernel table (compare profiles/r05_37/kernels_b2048.md).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_38; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv1x1_bn_gpu.py tests/test_bwd_fusion_gpu.py tests/test_conv1x1g_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for rep in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/step_$rep.log 2>&1 || { tail -20 $O/step_$rep.log; exit 1; }
echo "step_$rep $(grep '^{' $O/step_$rep.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --steps 6 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 400 --out $O/kernels.md > /dev/null
rm -rf $O/raw
head -2 $O/kernels.md | tail -1
grep -E "conv1x1_bn_fwd_kernel<.*, 3, [12]>" $O/kernels.md | cut -c1-200
