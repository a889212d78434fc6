#!/bin/bash
# GPU pass 42: stem wgrad with a real prefetch (unconditional loads, scalar wave index): tests, bench A/B, kernel times.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_stem_gpu.py tests/test_bn_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest42.log 2>&1; rc=$?
tail -25 gpurun_out/pytest42.log
[ $rc -eq 0 ] || exit $rc
for f in 1 0 1; do
CML_FUSE_STEM_CONV=$f timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-baseline --json-out gpurun_out/bench42_f$f.json > gpurun_out/bench42_f$f.log 2>&1 || exit $?
echo "stem=$f $(tail -1 gpurun_out/bench42_f$f.log | cut -c90-170)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace -d $R/gpurun_out/raw42 -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-baseline --profile-marker > $R/gpurun_out/prof42.log 2>&1 || exit $?
db=$(find $R/gpurun_out/raw42 -name '*.db' -print -quit)
python3 $R/tools/prof_summary.py "$db" --after spin_kernel --steps 6 --top 70 --out $R/gpurun_out/prof42_resnet_kernels.md
rm -rf $R/gpurun_out/raw42
grep -i "stem\|maxpool\|pad_c4" $R/gpurun_out/prof42_resnet_kernels.md | cut -c1-200
