#!/bin/bash
# Round 2, GPU pass 33: conv1x1 link / BN-backward-sums epilogue with batched operand loads --
# numerics, kernel bandwidth at the ResNet-50 shapes, bench, step profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out
rm -rf $O/r02_33_* $O/raw33
timeout -k 10 400 python -u -m pytest tests/test_conv1x1_bn_gpu.py tests/test_bwd_fusion_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r02_33_pytest.log 2>&1 || { tail -30 $O/r02_33_pytest.log; exit 1; }
tail -1 $O/r02_33_pytest.log
timeout -k 10 300 python -u bench/link_kernels.py > $O/r02_33_link.jsonl 2>$O/r02_33.err || { tail -20 $O/r02_33.err; exit 1; }
cat $O/r02_33_link.jsonl
for i in 1 2; do
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-baseline --virtual-workers 0 > $O/r02_33_bench$i.log 2>&1 || { tail -20 $O/r02_33_bench$i.log; exit 1; }
echo "run $i $(grep -o '"ms_per_step": [0-9.]*' $O/r02_33_bench$i.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw33 -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-baseline --virtual-workers 0 --profile-marker > $O/r02_33_prof.log 2>&1 || { tail -20 $O/r02_33_prof.log; exit 1; }
db=$(find $O/raw33 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 90 --out $O/r02_33_kernels.md
rm -rf $O/raw33
python3 $R/tools/kernel_classes.py $O/r02_33_kernels.md
grep "true, 1, 1\|true, 2, 1\|true, 1, 2\|true, 2, 2" $O/r02_33_kernels.md | cut -c1-60,100-200
