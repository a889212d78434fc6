#!/bin/bash
# r05 pass 19: stem weight gradient as a per-SIMD staging / MFMA ping-pong (tests, b2048 table);
# the 256 x 128 prologue routing fix; batch-256 kernel table and launch count.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_19; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem_gpu.py tests/test_wgrad1x1_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-baseline --b256-batch 0 --virtual-workers 0 > $O/bench_b2048.log 2>&1 || { tail -20 $O/bench_b2048.log; exit 1; }
grep '^{' $O/bench_b2048.log | cut -c1-220
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/bench.py --steps 6 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
db=$(find $O/raw -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 400 --out $O/kernels_b2048.md
python3 $R/tools/kernel_classes.py $O/kernels_b2048.md > $O/classes_b2048.md || true
rm -rf $O/raw
head -3 $O/kernels_b2048.md; cat $O/classes_b2048.md; grep -n "stem_wgrad_kernel" $O/kernels_b2048.md | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw256 -o run -- python3 $R/bench.py --batch 256 --steps 10 --warmup 3 --no-baseline --b256-batch 0 --virtual-workers 0 --profile-marker > $O/prof256.log 2>&1 || { tail -20 $O/prof256.log; exit 1; }
db=$(find $O/raw256 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 10 --top 500 --out $O/kernels_b256.md
python3 $R/tools/kernel_classes.py $O/kernels_b256.md > $O/classes_b256.md || true
rm -rf $O/raw256
head -3 $O/kernels_b256.md; cat $O/classes_b256.md
